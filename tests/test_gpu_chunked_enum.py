"""GPU parity of the enumerating finders in the chunked mode (more than 2^32 seed-mers):
MemHash / MaskedMemHash with enumeration tolerance > 1 (MemHash::EnumerateMatches,
MemHash.cpp:139-162, odometer MatchFinder.cpp:342-393) and PairwiseMatchFinder
(PairwiseMatchFinder.cpp:37-73).  Each resident chunk's groups are enumerated into probe rows
(mums_capi.hip run_pipeline_chunked, pairwise.hip launch_chunk_pairs + the enumeration kernels)
instead of the probe stage.

The chunked mode is forced on small inputs (MUMS_DEV_CHUNK_RECORDS caps the records per chunk,
as in tests/test_gpu_chunked_restart.py).  The MatchList, probe rows (AddHashEntry calls) and
collisions must equal the oracle's and the unchunked GPU run's.  Parity for these finders rests
on the oracle (no reference fixture covers them; its MemHash core is pinned by SURVEY App. C)."""
import os

import numpy as np
import pytest

from tests import repeat_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture
def force_chunks():
    def _set(cap):
        os.environ["MUMS_DEV_CHUNK_RECORDS"] = str(cap)
    yield _set
    os.environ.pop("MUMS_DEV_CHUNK_RECORDS", None)


def run_gpu(lm, seqs, seed, cls, rt, et, mask=0, start_points=None):
    with getattr(lm, cls)(0) as mh:
        mh.SetSeed(seed)
        if cls != "PairwiseMatchFinder":
            mh.SetRepeatTolerance(rt)
            mh.SetEnumerationTolerance(et)
        if cls == "MaskedMemHash":
            mh.SetMask(mask)
        ml = mh.FindMatches(seqs) if start_points is None else mh.FindMatchesFromPosition(seqs, start_points)
        return ml, mh.stats()


def check(lm, oracle_mod, force_chunks, seqs, w, cls="MemHash", rt=0, et=1, mask=0, chunks=4, start_points=None):
    seed = oracle_mod.get_seed(w)
    ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, seed, repeat_tol=rt, enum_tol=et,
                                                       masked=cls == "MaskedMemHash", seq_mask=mask,
                                                       pairwise=cls == "PairwiseMatchFinder",
                                                       start_points=start_points)
    flat_ml, flat = run_gpu(lm, seqs, seed, cls, rt, et, mask, start_points)
    n = sum(len(s) for s in seqs)
    cap = max(n // chunks, 4096)
    while True:   # N gaps put many records into the all-A key's MSD digit: a chunk must hold it
        force_chunks(cap)
        try:
            ml, st = run_gpu(lm, seqs, seed, cls, rt, et, mask, start_points)
            break
        except lm.MumsError as e:
            if "one MSD digit" not in str(e) or cap > n:
                raise
            cap *= 2
    assert st["chunks"] >= 2
    assert st["probes"] == ref["probes"] == flat["probes"] > 0, (st["probes"], ref["probes"], flat["probes"])
    assert st["restarts"] == ref["restarts"]
    assert len(ml) == len(ref_len) == len(flat_ml), (len(ml), len(ref_len), len(flat_ml))
    assert (ml.lengths == ref_len).all() and (ml.starts == ref_starts).all()
    assert st["collision_count"] == ref["collision_count"]
    return st, ref


@pytest.mark.parametrize("w", [16, 19, 21])
@pytest.mark.parametrize("rt,et", [(1, 2), (2, 3)])
def test_enumeration_tolerance_chunked(gpu_lib, oracle_mod, force_chunks, w, rt, et):
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=40, tandem=False, seed=w + et)
    check(gpu_lib, oracle_mod, force_chunks, seqs, w, rt=rt, et=et)


@pytest.mark.parametrize("rt,et", [(39, 12), (8, 9)])
def test_enumeration_walk_kernels_chunked(gpu_lib, oracle_mod, force_chunks, rt, et):
    """enum_tol above the slot kernels' bound (pairwise.hip en_*_walk_kernel) over chunks."""
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=40, tandem=False, seed=et)
    check(gpu_lib, oracle_mod, force_chunks, seqs, 17, rt=rt, et=et, chunks=6)


@pytest.mark.parametrize("mask", [0, 5])
def test_masked_enumeration_chunked(gpu_lib, oracle_mod, force_chunks, mask):
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=40, tandem=False, seed=50 + mask)
    check(gpu_lib, oracle_mod, force_chunks, seqs, 18, cls="MaskedMemHash", rt=39, et=3, mask=mask)


@pytest.mark.parametrize("w", [16, 19, 21])
def test_pairwise_chunked(gpu_lib, oracle_mod, force_chunks, w):
    seqs = oracle_mod.generate(5, 40_000, 0.03, 600 + w)
    check(gpu_lib, oracle_mod, force_chunks, seqs, w, cls="PairwiseMatchFinder", chunks=5)


def test_pairwise_chunked_repeats(gpu_lib, oracle_mod, force_chunks):
    seqs = repeat_inputs.high_copy(G=4, n=50_000, copies=30, tandem=False, seed=7)
    check(gpu_lib, oracle_mod, force_chunks, seqs, 17, cls="PairwiseMatchFinder")


def test_enumeration_with_restarts_chunked(gpu_lib, oracle_mod, force_chunks):
    """MER_REPEAT_LIMIT restarts (chunked_restart) before the chunks are enumerated."""
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    st, ref = check(gpu_lib, oracle_mod, force_chunks, seqs, 17, rt=1, et=2)
    assert ref["restarts"] > 0


def test_pairwise_with_restarts_chunked(gpu_lib, oracle_mod, force_chunks):
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=2)
    st, ref = check(gpu_lib, oracle_mod, force_chunks, seqs, 16, cls="PairwiseMatchFinder")
    assert ref["restarts"] > 0


def test_enumeration_start_points_chunked(gpu_lib, oracle_mod, force_chunks):
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=40, tandem=False, seed=3)
    check(gpu_lib, oracle_mod, force_chunks, seqs, 17, rt=2, et=2, start_points=[1000, 25_000, 7])
