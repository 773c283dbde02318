"""MatchFinder::LogProgress (MatchFinder.cpp:55-56, 137-164, 296-309): the "N%.." text the
reference's merge writes at every whole percent of the mers (counted at each 10 000-mer buffer
refill, a newline every ten), restated by the GPU from the SML keys at the buffer ends and the
restart plan's consumed positions, against the oracle's literal SearchRange, byte for byte."""
import os

import pytest

from tests import repeat_inputs

pytestmark = pytest.mark.gpu


def gpu_progress(lm, seqs, seed, cls="MemHash", mask=0, start_points=None):
    with getattr(lm, cls)(0) as mh:
        mh.SetSeed(seed)
        if cls == "MaskedMemHash":
            mh.SetMask(mask)
        mh.LogProgress(True)
        if start_points is None:
            mh.FindMatches(seqs)
        else:
            mh.FindMatchesFromPosition(seqs, start_points)
        return mh.ProgressLog(), mh.stats()


def check(lm, oracle_mod, seqs, w=15, cls="MemHash", mask=0, start_points=None):
    seed = oracle_mod.get_seed(w)
    text, st = gpu_progress(lm, seqs, seed, cls, mask, start_points)
    _, _, ref = oracle_mod.find_matches(seqs, seed, masked=cls == "MaskedMemHash", seq_mask=mask,
                                        start_points=start_points)
    assert st["restarts"] == ref["restarts"]
    assert text == ref["progress"]
    return text, ref


@pytest.mark.parametrize("G,n,p,w", [(3, 2_000_000, 0.01, 15), (2, 1_000_000, 1.0, 15), (5, 300_000, 0.02, 13),
                                     (4, 1_500_000, 0.01, 19), (3, 1_000_000, 0.01, 21), (2, 9_999, 0.01, 11)])
def test_progress_plain(gpu_lib, oracle_mod, G, n, p, w):
    text, _ = check(gpu_lib, oracle_mod, oracle_mod.generate(G, n, p, 70 + G), w)
    # total = sequence lengths (MatchFinder.cpp:146): the last L-1 bases of a linear genome hold no
    # mer, so the text stops at 99%
    assert (text.endswith("99%..") and "100%" not in text) or n < 100_000


def test_progress_masked(gpu_lib, oracle_mod):
    check(gpu_lib, oracle_mod, oracle_mod.generate(4, 400_000, 0.02, 3), 15, "MaskedMemHash", 0b1011)


@pytest.mark.parametrize("sp", [[0, 0, 0], [1000, 25_000, 7], [150_000, 0, 190_000], [9_990, 19_990, 29_990]])
def test_progress_start_points(gpu_lib, oracle_mod, sp):
    check(gpu_lib, oracle_mod, oracle_mod.generate(3, 200_000, 0.02, 777), 15, start_points=sp)


@pytest.mark.parametrize("seed", range(3))
def test_progress_restarts_n_gapped(gpu_lib, oracle_mod, seed):
    seqs = repeat_inputs.n_gapped(G=3, n=300_000, gaps=((40_000, 3000), (120_000, 3000), (250_000, 4000)),
                                  shift=500 + 100 * seed, seed=seed)
    _, ref = check(gpu_lib, oracle_mod, seqs, 15)
    assert ref["restarts"] > 0


def test_progress_restarts_high_copy(gpu_lib, oracle_mod):
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=2000, seed=2)
    _, ref = check(gpu_lib, oracle_mod, seqs, 15)
    assert ref["restarts"] > 0


def test_progress_restarts_with_start_points(gpu_lib, oracle_mod):
    seqs = repeat_inputs.n_gapped(G=3, n=90_000, gaps=((2_000, 25_000), (60_000, 4_000)), shift=1_300, seed=31)
    check(gpu_lib, oracle_mod, seqs, 19, start_points=[1000, 25_000, 7])


@pytest.mark.parametrize("gapped", [False, True])
def test_progress_chunked_mode(gpu_lib, oracle_mod, monkeypatch, gapped):
    """the chunked mode (> 2^32 seed-mers) forced on a small input: same text"""
    seqs = (repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
            if gapped else oracle_mod.generate(3, 300_000, 0.02, 99))
    n = sum(len(s) for s in seqs)
    monkeypatch.setenv("MUMS_DEV_CHUNK_RECORDS", str(max(n // 2, 4096) if not gapped else n // 2 + 20_000))
    seed = oracle_mod.get_seed(19)
    text, st = gpu_progress(gpu_lib, seqs, seed)
    _, _, ref = oracle_mod.find_matches(seqs, seed)
    assert st["chunks"] >= 2
    assert text == ref["progress"]


@pytest.mark.parametrize("w,gapped", [(23, False), (25, False), (23, True)])
def test_progress_pair_path(gpu_lib, oracle_mod, w, gapped):
    """the pair-key path (seed weight > 21): keys restated from the key-order ranks"""
    seqs = (repeat_inputs.n_gapped(G=3, n=250_000, gaps=((40_000, 3000), (150_000, 3000)), shift=600, seed=5)
            if gapped else oracle_mod.generate(3, 600_000, 0.01, 23))
    _, ref = check(gpu_lib, oracle_mod, seqs, w)
    if gapped:
        assert ref["restarts"] > 0


@pytest.mark.parametrize("w,gapped", [(15, False), (23, False), (15, True)])
def test_progress_pairwise(gpu_lib, oracle_mod, w, gapped):
    """PairwiseMatchFinder searches with MatchFinder::FindMatchSeeds (PairwiseMatchFinder.cpp:
    37-73 only changes how a seed group is hashed), so its text is the same merge's"""
    seqs = (repeat_inputs.n_gapped(G=3, n=250_000, gaps=((40_000, 3000), (150_000, 3000)), shift=600, seed=6)
            if gapped else oracle_mod.generate(4, 400_000, 0.02, 41))
    seed = oracle_mod.get_seed(w)
    text, st = gpu_progress(gpu_lib, seqs, seed, "PairwiseMatchFinder")
    _, _, ref = oracle_mod.find_matches(seqs, seed, pairwise=True)
    assert st["restarts"] == ref["restarts"]
    assert text == ref["progress"] and text
