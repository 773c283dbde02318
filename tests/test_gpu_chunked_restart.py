"""GPU parity of MER_REPEAT_LIMIT restarts (MatchFinder.cpp:253-277) and FindMatchesFromPosition
start points (MemHash.cpp:117-127) in the chunked mode (more than 2^32 seed-mers; chunked.hip's
chunked_restart over the resident chunks), against the oracle's literal SearchRange with the
std::sort SortedMerList order (MemorySML.cpp:54).

The chunked mode is forced on small inputs (MUMS_DEV_CHUNK_RECORDS caps the records per chunk):
the same inputs as tests/test_gpu_restart.py and tests/tie_inputs.py (N gaps, high-copy repeats,
start points inside runs of equal keys), at the seed weights the chunked mode runs (16-19).
MatchList, collisions, restarts and the offset log must equal the oracle's; the count of
groups above MER_REPEAT_LIMIT must equal the unchunked run's."""
import os

import numpy as np
import pytest

from tests import repeat_inputs, tie_inputs

pytestmark = pytest.mark.gpu


@pytest.fixture
def force_chunks():
    def _set(cap, stream=False):
        os.environ["MUMS_DEV_CHUNK_RECORDS"] = str(cap)
        if stream:
            os.environ["MUMS_DEV_CHUNK_STREAM"] = "1"
    yield _set
    os.environ.pop("MUMS_DEV_CHUNK_RECORDS", None)
    os.environ.pop("MUMS_DEV_CHUNK_STREAM", None)


def run_gpu(lm, seqs, seed, cls="MemHash", mask=0, start_points=None):
    with getattr(lm, cls)(0) as mh:
        mh.SetSeed(seed)
        if cls == "MaskedMemHash":
            mh.SetMask(mask)
        if start_points is None:
            ml = mh.FindMatches(seqs)
        else:
            ml = mh.FindMatchesFromPosition(seqs, start_points)
        return ml, mh.stats(), mh.OffsetLog()


def check(lm, oracle_mod, force_chunks, seqs, w, chunks=4, cls="MemHash", mask=0, start_points=None):
    seed = oracle_mod.get_seed(w)
    ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, seed, masked=cls == "MaskedMemHash", seq_mask=mask,
                                                       start_points=start_points)
    _, flat, _ = run_gpu(lm, seqs, seed, cls, mask, start_points)
    n = sum(len(s) for s in seqs)
    cap = max(n // chunks, 4096)
    while True:   # N gaps put many records into the all-A key's MSD digit: a chunk must hold it
        force_chunks(cap)
        try:
            ml, st, offlog = run_gpu(lm, seqs, seed, cls, mask, start_points)
            break
        except lm.MumsError as e:
            if "one MSD digit" not in str(e) or cap > n:
                raise
            cap *= 2
    assert st["chunks"] >= 2
    assert st["restarts"] == ref["restarts"], (st["restarts"], ref["restarts"])
    assert np.array_equal(offlog, ref["offset_log"])
    assert len(ml) == len(ref_len), (len(ml), len(ref_len))
    assert (ml.lengths == ref_len).all() and (ml.starts == ref_starts).all()
    assert st["collision_count"] == ref["collision_count"]
    assert st["repeat_limit_groups"] == flat["repeat_limit_groups"]
    return st, ref


@pytest.mark.parametrize("cls,mask", [("MemHash", 0), ("MaskedMemHash", 7)])
@pytest.mark.parametrize("w", [16, 19, 21])
def test_n_gapped(gpu_lib, oracle_mod, force_chunks, cls, mask, w):
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    st, ref = check(gpu_lib, oracle_mod, force_chunks, seqs, w, cls=cls, mask=mask)
    assert ref["restarts"] > 0


@pytest.mark.parametrize("tandem", [False, True])
def test_high_copy(gpu_lib, oracle_mod, force_chunks, tandem):
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=2000, tandem=tandem, seed=2)
    check(gpu_lib, oracle_mod, force_chunks, seqs, 17, chunks=6)


def test_runs_across_buffer_boundaries(gpu_lib, oracle_mod, force_chunks):
    seqs = repeat_inputs.n_gapped(G=4, n=90_000, gaps=((2_000, 25_000), (60_000, 10_022)), shift=1_300, seed=13)
    check(gpu_lib, oracle_mod, force_chunks, seqs, 18, chunks=8)


@pytest.mark.parametrize("seed", list(range(0, 12)) + [95, 106])
def test_mixed_repeats_fuzz(gpu_lib, oracle_mod, force_chunks, seed):
    check(gpu_lib, oracle_mod, force_chunks, repeat_inputs.mixed_repeats(seed), 16 + seed % 4, chunks=3 + seed % 5)


@pytest.mark.parametrize("seed", range(6))
def test_multi_gap_ties(gpu_lib, oracle_mod, force_chunks, seed):
    # restarts at the "A...AC" gap keys: start points inside runs of equal full keys
    check(gpu_lib, oracle_mod, force_chunks, tie_inputs.multi_gap(seed=seed), 16 + seed % 4)


@pytest.mark.parametrize("sp", [[0, 0, 0], [1000, 25_000, 7], [50_000, 0, 59_000]])
def test_start_points_plain(gpu_lib, oracle_mod, force_chunks, sp):
    seqs = oracle_mod.generate(3, 60_000, 0.02, 777)
    check(gpu_lib, oracle_mod, force_chunks, seqs, 17, start_points=sp)


@pytest.mark.parametrize("sp", [[1000, 25_000, 7], [3, 9_999, 10_001, 40_000]])
def test_start_points_with_restarts(gpu_lib, oracle_mod, force_chunks, sp):
    seqs = repeat_inputs.n_gapped(G=len(sp), n=90_000, gaps=((2_000, 25_000), (60_000, 4_000)), shift=1_300,
                                  seed=31)
    check(gpu_lib, oracle_mod, force_chunks, seqs, 19, start_points=sp)


@pytest.mark.parametrize("w", [20, 21])
def test_w2x_start_points_with_restarts(gpu_lib, oracle_mod, force_chunks, w):
    """w20-21: the full keys of the restart plan take their top bits from the split buckets."""
    seqs = repeat_inputs.n_gapped(G=3, n=90_000, gaps=((2_000, 25_000), (60_000, 4_000)), shift=1_300, seed=33)
    check(gpu_lib, oracle_mod, force_chunks, seqs, w, start_points=[1000, 25_000, 7])


@pytest.mark.parametrize("sd", range(4))
def test_start_points_in_duplicate_runs(gpu_lib, oracle_mod, force_chunks, sd):
    # genome 1 holds a second copy of a block: its start point splits runs of two equal keys
    rng = np.random.default_rng(200 + sd)
    seqs = tie_inputs.dup_block(seed=80 + sd)
    sp = [int(rng.integers(0, 30_000)), int(rng.integers(1, 50_000)), 0]
    check(gpu_lib, oracle_mod, force_chunks, seqs, 16 + sd, start_points=sp)


def test_streaming_layout_refuses_start_points(gpu_lib, oracle_mod, force_chunks):
    seqs = oracle_mod.generate(3, 60_000, 0.02, 3)
    force_chunks(50_000, stream=True)
    with pytest.raises(gpu_lib.MumsError) as ei:
        run_gpu(gpu_lib, seqs, oracle_mod.get_seed(17), start_points=[5, 6, 7])
    assert ei.value.code == gpu_lib.MUMS_E_UNSUPPORTED


def test_tie_workspace_kept_across_seed_stage_calls(gpu_lib, oracle_mod, force_chunks):
    """Seed-stage-only chunked runs keep the tie workspace (keep_tiebuf, mums_capi.hip); the
    FindMatches calls after them reuse it: the same MatchList as the oracle every time."""
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    seed = oracle_mod.get_seed(19)
    ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, seed)
    assert ref["restarts"] > 0
    force_chunks(sum(len(s) for s in seqs) // 2 + 20_000)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        for s in seqs:
            mh.AddSequence(s)
        for _ in range(2):
            mh.FindStage(gpu_lib.STAGE_SEEDS)
        for _ in range(2):
            ml = mh.FindMatches()
            st = mh.stats()
            assert st["chunks"] >= 2 and st["restarts"] == ref["restarts"]
            assert (ml.lengths == ref_len).all() and (ml.starts == ref_starts).all()
        mh.FindStage(gpu_lib.STAGE_SEEDS)
        assert (mh.FindMatches().starts == ref_starts).all()


# repeat tolerance in the chunked mode (MemHash.cpp:139-162): the first copies of a genome in
# SortedMerList order, i.e. every run of equal keys in std::sort order (chunked_tie_fix)
RTOL_CASES = {k: v for k, v in tie_inputs.CASES.items()
              if v[1].get("repeat_tol", 0) > 0 and v[1].get("enum_tol", 1) == 1}


@pytest.mark.parametrize("name", sorted(RTOL_CASES))
@pytest.mark.parametrize("chunks", [2, 4])   # (w17: 16 implicit digits, repeats fill some)
def test_repeat_tolerance_chunked(gpu_lib, oracle_mod, force_chunks, name, chunks):
    gen, opts = RTOL_CASES[name]
    seqs = gen()
    w = max(opts.get("w", 15), 17)   # the chunked mode's weights: 2w + 1 > 32
    seed = oracle_mod.get_seed(w)
    with oracle_mod.sml_tie_rule("std"):
        ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, seed, repeat_tol=opts["repeat_tol"])
    force_chunks(max(sum(len(s) for s in seqs) // chunks, 4096))
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        mh.SetRepeatTolerance(opts["repeat_tol"])
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert st["chunks"] >= 2
    assert len(ml) == len(ref_len), (len(ml), len(ref_len))
    assert (ml.lengths == ref_len).all() and (ml.starts == ref_starts).all()
    assert st["collision_count"] == ref["collision_count"]
    assert st["restarts"] == ref["restarts"]


@pytest.mark.parametrize("rtol", [1, 3])
def test_repeat_tolerance_chunked_with_restarts(gpu_lib, oracle_mod, force_chunks, rtol):
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    seed = oracle_mod.get_seed(17)
    with oracle_mod.sml_tie_rule("std"):
        ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, seed, repeat_tol=rtol)
    assert ref["restarts"] > 0
    force_chunks(max(sum(len(s) for s in seqs) // 4, 4096))
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        mh.SetRepeatTolerance(rtol)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
        offlog = mh.OffsetLog()
    assert st["chunks"] >= 2
    assert (ml.lengths == ref_len).all() and (ml.starts == ref_starts).all() and len(ml) == len(ref_len)
    assert st["restarts"] == ref["restarts"] and np.array_equal(offlog, ref["offset_log"])
    assert st["collision_count"] == ref["collision_count"]
