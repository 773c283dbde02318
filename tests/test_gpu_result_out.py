"""MemHash::GetMatchList into caller-owned host buffers (pinned memory reused across calls,
the end-to-end bench's form): the same MatchList as the default copy; wrong buffers refused."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_get_match_list_into_pinned_buffers(gpu_lib, oracle_mod):
    import torch
    seqs = oracle_mod.generate(3, 200_000, 0.02, 5)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(15))
        ref = mh.FindMatches(seqs)
        n = len(ref)
        out = (torch.empty(n + 7, dtype=torch.int64, pin_memory=True).numpy().view(np.uint64),
               torch.empty((n + 7) * 3, dtype=torch.int64, pin_memory=True).numpy())
        ml = mh.GetMatchList(out)
        assert np.array_equal(ml.lengths, ref.lengths) and np.array_equal(ml.starts, ref.starts)
        with pytest.raises(ValueError):
            mh.GetMatchList((np.zeros(n - 1, dtype=np.uint64), np.zeros(n * 3, dtype=np.int64)))
        with pytest.raises(ValueError):
            mh.GetMatchList((np.zeros(n, dtype=np.int64), np.zeros(n * 3, dtype=np.int64)))
