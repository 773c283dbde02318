"""EliminateOverlaps (Aligner.cpp:62-176) on the GPU against the oracle's restatement
(oracle/eliminate_overlaps.c, whose std::sort replay is pinned to this toolchain's real
std::sort by tests/test_eliminate_overlaps_cpu.py): the device replay of libstdc++'s
introsort alone, random MatchLists with overlaps / ties / reverse components, and the
MatchLists of BASELINE configs 2 and 4 (known-answer inputs, md5-checked first)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from test_eliminate_overlaps_cpu import random_matchlist

pytestmark = pytest.mark.gpu

CASES = {(c["G"], c["n"], c["p"], c["mode"]): c for c in json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["cases"]}


@pytest.mark.parametrize("n", [0, 1, 16, 17, 100, 1000, 65536, 300000])
@pytest.mark.parametrize("span", [1, 4, 1000, 1 << 40])
def test_std_sort_replay(gpu_lib, oracle_mod, n, span):
    rng = np.random.default_rng(n + span % 977)
    keys = rng.integers(0, span, size=n, dtype=np.uint64)
    if n > 10:
        keys[rng.integers(0, n, size=n // 4)] = 0
    with gpu_lib.MemHash(0) as mh:
        got = mh._debug_std_sort(keys)
    assert np.array_equal(got, oracle_mod.std_sort_ids(keys))


@pytest.mark.parametrize("depth", [0, 1, 3])
@pytest.mark.parametrize("n", [40, 5000])
def test_std_sort_replay_depth_limit(gpu_lib, oracle_mod, depth, n):
    rng = np.random.default_rng(depth * 10 + n)
    keys = rng.integers(0, 30, size=n, dtype=np.uint64)
    with gpu_lib.MemHash(0) as mh:
        got = mh._debug_std_sort(keys, depth)
    assert np.array_equal(got, oracle_mod.std_sort_ids(keys, depth))


def eo_both(gpu_lib, oracle_mod, lengths, starts):
    ml = gpu_lib.MatchList(np.asarray(lengths, dtype=np.uint64), np.asarray(starts, dtype=np.int64))
    got = gpu_lib.EliminateOverlaps(ml)
    rl, rs = oracle_mod.eliminate_overlaps(lengths, starts)
    return got, rl, rs


@pytest.mark.parametrize("M,G,span,seed", [(2, 2, 50, 1), (10, 2, 100, 2), (200, 3, 2000, 3), (3000, 4, 30000, 4),
                                           (5000, 8, 20000, 5), (20000, 5, 400000, 6), (3000, 3, 300, 7),
                                           (200000, 4, 4000000, 8)])
def test_eliminate_overlaps_random(gpu_lib, oracle_mod, M, G, span, seed):
    rng = np.random.default_rng(seed)
    lengths, starts = random_matchlist(rng, M, G, start_span=span)
    got, rl, rs = eo_both(gpu_lib, oracle_mod, lengths, starts)
    assert len(got) == len(rl)
    assert np.array_equal(got.lengths, rl) and np.array_equal(got.starts, rs)


@pytest.mark.parametrize("key", [(4, 10_000_000, 0.01, "MemHash"), (4, 10_000_000, 1.0, "MemHash"),
                                 (3, 5_000_000, 0.01, "MaskedMemHash"), (3, 5_000_000, 1.0, "MaskedMemHash")],
                         ids=["c2_related", "c2_iid", "c4_related", "c4_iid"])
def test_eliminate_overlaps_on_baseline_matchlists(gpu_lib, oracle_mod, key):
    c = CASES[key]
    seqs = oracle_mod.generate(c["G"], c["n"], c["p"], 12345)
    cls = gpu_lib.MaskedMemHash if c["mode"] == "MaskedMemHash" else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(c["w"]))
        if c["mode"] == "MaskedMemHash":
            mh.SetMask(c.get("mask", 0))
        ml = mh.FindMatches(seqs)
        assert hashlib.md5(ml.text().encode()).hexdigest() == c["md5"]
        mh.EliminateOverlaps()   # on the device-resident MatchList
        got = mh.GetMatchList()
    rl, rs = oracle_mod.eliminate_overlaps(ml.lengths, ml.starts)
    assert len(got) == len(rl)
    assert np.array_equal(got.lengths, rl) and np.array_equal(got.starts, rs)
