"""GPU parity of MatchFinder::SearchRange's MER_REPEAT_LIMIT restart (MatchFinder.cpp:253-277)
and of FindMatchesFromPosition (MemHash.cpp:117-127): the HIP path (restart.hip fix-up of the
merged stream) against the oracle's literal SearchRange, bit for bit, on N-gapped assemblies
(N encodes as A: one all-A key group per gap) and high-copy repeats."""
import numpy as np
import pytest

from tests import repeat_inputs

pytestmark = pytest.mark.gpu


def run_gpu(lm, seqs, seed, cls="MemHash", mask=0, start_points=None, repeat_tol=0, enum_tol=1):
    with getattr(lm, cls)(0) as mh:
        mh.SetSeed(seed)
        mh.SetRepeatTolerance(repeat_tol)
        mh.SetEnumerationTolerance(enum_tol)
        if cls == "MaskedMemHash":
            mh.SetMask(mask)
        if start_points is None:
            ml = mh.FindMatches(seqs)
        else:
            ml = mh.FindMatchesFromPosition(seqs, start_points)
        return ml, mh.stats(), mh.OffsetLog()


def check(lm, oracle_mod, seqs, w=15, cls="MemHash", mask=0, start_points=None, repeat_tol=0, enum_tol=1,
          need_restart=True):
    seed = oracle_mod.get_seed(w)
    ml, st, offlog = run_gpu(lm, seqs, seed, cls, mask, start_points, repeat_tol, enum_tol)
    ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, seed, repeat_tol=repeat_tol, enum_tol=enum_tol,
                                                       masked=cls == "MaskedMemHash", seq_mask=mask,
                                                       pairwise=cls == "PairwiseMatchFinder",
                                                       start_points=start_points)
    assert st["restarts"] == ref["restarts"], (st["restarts"], ref["restarts"])
    assert np.array_equal(offlog, ref["offset_log"])
    assert len(ml) == len(ref_len)
    assert (ml.lengths == ref_len).all()
    assert (ml.starts == ref_starts).all()
    assert st["collision_count"] == ref["collision_count"]
    if need_restart:
        assert st["repeat_limit_groups"] > 0 and ref["restarts"] > 0
    return st, ref


@pytest.mark.parametrize("cls,mask", [("MemHash", 0), ("MaskedMemHash", 7)])
def test_n_gapped_3000(gpu_lib, oracle_mod, cls, mask):
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    check(gpu_lib, oracle_mod, seqs, cls=cls, mask=mask)


@pytest.mark.parametrize("cls,mask", [("MemHash", 0), ("MaskedMemHash", 7)])
@pytest.mark.parametrize("tandem", [False, True])
def test_high_copy_2000(gpu_lib, oracle_mod, cls, mask, tandem):
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=2000, tandem=tandem, seed=2)
    check(gpu_lib, oracle_mod, seqs, cls=cls, mask=mask)


def test_high_copy_single_genome(gpu_lib, oracle_mod):
    seqs = repeat_inputs.high_copy(G=3, n=30_000, copies=2000, only_genome=0, seed=5)
    check(gpu_lib, oracle_mod, seqs, need_restart=False)


@pytest.mark.parametrize("w", [17, 19, 21, 23])   # packed records with MSD bits (17-21), pair path (23)
def test_weights(gpu_lib, oracle_mod, w):
    seqs = repeat_inputs.n_gapped(G=4, n=80_000, gaps=((10_000, 3000), (50_000, 1800)), shift=300, seed=w)
    check(gpu_lib, oracle_mod, seqs, w=w)


def test_runs_across_buffer_boundaries(gpu_lib, oracle_mod):
    # N runs longer than MER_BUFFER_SIZE: collected in several steps, the check fires between them
    seqs = repeat_inputs.n_gapped(G=4, n=90_000, gaps=((2_000, 25_000), (60_000, 10_022)), shift=1_300, seed=13)
    check(gpu_lib, oracle_mod, seqs)


@pytest.mark.parametrize("seed", list(range(0, 24)) + [26, 95, 98, 99, 106])
def test_mixed_repeats_fuzz(gpu_lib, oracle_mod, seed):
    check(gpu_lib, oracle_mod, repeat_inputs.mixed_repeats(seed), need_restart=False)


def test_repeat_tolerance(gpu_lib, oracle_mod):
    seqs = repeat_inputs.high_copy(G=3, n=40_000, copies=1500, seed=17)
    check(gpu_lib, oracle_mod, seqs, repeat_tol=2)


def test_enumeration_tolerance(gpu_lib, oracle_mod):
    seqs = repeat_inputs.n_gapped(G=3, n=60_000, gaps=((20_000, 3000),), seed=23)
    check(gpu_lib, oracle_mod, seqs, repeat_tol=1, enum_tol=2)


def test_pairwise(gpu_lib, oracle_mod):
    seqs = repeat_inputs.n_gapped(G=3, n=60_000, gaps=((20_000, 3000),), seed=29)
    check(gpu_lib, oracle_mod, seqs, cls="PairwiseMatchFinder")


# ---- FindMatchesFromPosition (MemHash.cpp:117-127) ----------------------------------
@pytest.mark.parametrize("sp", [[0, 0, 0], [1000, 25_000, 7], [50_000, 0, 59_000]])
def test_start_points_plain(gpu_lib, oracle_mod, sp):
    seqs = oracle_mod.generate(3, 60_000, 0.02, 777)
    check(gpu_lib, oracle_mod, seqs, start_points=sp, need_restart=False)


@pytest.mark.parametrize("sp", [[1000, 25_000, 7], [3, 9_999, 10_001, 40_000]])
def test_start_points_with_restarts(gpu_lib, oracle_mod, sp):
    G = len(sp)
    seqs = repeat_inputs.n_gapped(G=G, n=90_000, gaps=((2_000, 25_000), (60_000, 4_000)), shift=1_300, seed=31)
    check(gpu_lib, oracle_mod, seqs, start_points=sp, need_restart=False)


def test_no_restart_path_untouched(gpu_lib, oracle_mod):
    # ordinary input: no group above 1000, nothing restarted, empty offset log
    seqs = oracle_mod.generate(3, 100_000, 0.02, 5)
    st, ref = check(gpu_lib, oracle_mod, seqs, need_restart=False)
    assert st["repeat_limit_groups"] == 0 and st["restarts"] == 0 and ref["restarts"] == 0


def test_start_points_count_must_match(gpu_lib, oracle_mod):
    # MatchFinder::FindMatchSeeds throws InvalidData unless there is one start point per
    # sequence (MatchFinder.cpp:197-199)
    seqs = oracle_mod.generate(3, 20_000, 0.02, 9)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(15))
        with pytest.raises(gpu_lib.MumsError) as ei:
            mh.FindMatchesFromPosition(seqs, [5, 7])
        assert ei.value.code == gpu_lib.MUMS_E_INVALID
