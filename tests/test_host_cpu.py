"""Host-side logic that needs no GPU: MatchList text form, seed helpers."""
import numpy as np

import libmems_amd as lm


def test_matchlist_text_format():
    ml = lm.MatchList(np.array([39940, 7], dtype=np.uint64), np.array([[1, 1], [-5, 0]], dtype=np.int64))
    assert ml.text() == "39940\t1\t1\n7\t-5\t0\n"
    assert len(ml) == 2


def test_seed_length_weight():
    assert lm.getSeedLength(0x7AC9AF) == 23 and lm.getSeedWeight(0x7AC9AF) == 15
    assert lm.getSeedLength(0x7B974EF) == 27 and lm.getSeedWeight(0x7B974EF) == 19
    assert lm.getSeedLength(0) == 0
