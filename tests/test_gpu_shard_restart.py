"""GPU parity of MER_REPEAT_LIMIT restarts (MatchFinder.cpp:253-277) and FindMatchesFromPosition
start points (MemHash.cpp:117-127) in the sharded mode (mums_shard_run, shard_comm.hip).  By
default every rank plans on its own part of every SortedMerList (restart_plan.h's distributed
PlanData, rank after rank with the running start points), the runs a start point falls into
get their std::sort order (MemorySML.cpp:54) on rank g % world, and every rank compacts its
own live records (mums_shard_restart_counts .. _finish).  MUMS_DEV_SHARD_RESTART=gather forces
the fallback: the streams gathered onto rank 0, which plans on the whole stream.

Ranks are threads of one process over the host-staged communicator (one GPU); genome blocks
and position slices.  MatchList, collisions (summed over ranks), restarts and the offset log
must equal the oracle's."""
import os

import numpy as np
import pytest

from tests import repeat_inputs, tie_inputs

pytestmark = pytest.mark.gpu


PATHS = {"local": 0, "gather": 0}   # restarts planned per path (reported by test_zz_path_counts)


def check(lm, oracle_mod, seqs, world, w=15, layout="blocks", start_points=None, table_size=40000, info=None,
          repeat_tol=0, enum_tol=1):
    if layout == "slices":   # world / G position slices per genome
        world = len(seqs) * (1 if world <= len(seqs) else 2)
    seed = oracle_mod.get_seed(w)
    with oracle_mod.sml_tie_rule("std"):
        ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, seed, start_points=start_points,
                                                           table_size=table_size, repeat_tol=repeat_tol,
                                                           enum_tol=enum_tol)
    with lm.ShardedMemHash([0] * world, comm="local", layout=layout, table_size=table_size) as sh:
        sh.SetSeed(seed)
        sh.SetRepeatTolerance(repeat_tol)
        sh.SetEnumerationTolerance(enum_tol)
        if start_points is None:
            ml = sh.FindMatches(seqs)
        else:
            ml = sh.FindMatchesFromPosition(seqs, start_points)
        stats = sh.stats_per_rank
        offlog = sh.OffsetLog()
        rinfo = sh.restart_info
    if info is not None:
        info.extend(rinfo)
    paths = {i["path"] for i in rinfo}
    assert len(paths) == 1, rinfo   # every rank took the same path
    if 1 in paths:
        PATHS["local"] += 1
    if 2 in paths:
        PATHS["gather"] += 1
    assert all(s["restarts"] == ref["restarts"] for s in stats), ([s["restarts"] for s in stats], ref["restarts"])
    assert np.array_equal(offlog, ref["offset_log"])
    assert len(ml) == len(ref_len), (len(ml), len(ref_len))
    assert np.array_equal(ml.lengths, ref_len) and np.array_equal(ml.starts, ref_starts)
    assert sum(s["collision_count"] for s in stats) == ref["collision_count"]
    return ref


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("layout", ["blocks", "slices"])
def test_n_gapped(gpu_lib, oracle_mod, world, layout):
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    ref = check(gpu_lib, oracle_mod, seqs, world, layout=layout)
    assert ref["restarts"] > 0


@pytest.mark.parametrize("tandem", [False, True])
@pytest.mark.parametrize("world", [2, 4])
def test_high_copy(gpu_lib, oracle_mod, tandem, world):
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=2000, tandem=tandem, seed=2)
    check(gpu_lib, oracle_mod, seqs, world)


def test_runs_across_buffer_boundaries(gpu_lib, oracle_mod):
    seqs = repeat_inputs.n_gapped(G=4, n=90_000, gaps=((2_000, 25_000), (60_000, 10_022)), shift=1_300, seed=13)
    check(gpu_lib, oracle_mod, seqs, 3, w=17, layout="slices")


@pytest.mark.parametrize("seed", list(range(0, 10)) + [95, 106])
def test_mixed_repeats_fuzz(gpu_lib, oracle_mod, seed):
    check(gpu_lib, oracle_mod, repeat_inputs.mixed_repeats(seed), 2 + seed % 3,
          layout="slices" if seed % 2 else "blocks")


@pytest.mark.parametrize("seed", range(6))
def test_multi_gap_ties(gpu_lib, oracle_mod, seed):
    # restarts at the "A...AC" gap keys: start points inside runs of equal full keys
    check(gpu_lib, oracle_mod, tie_inputs.multi_gap(seed=seed), 2 + seed % 3, w=15 + 2 * (seed % 3))


def test_small_table(gpu_lib, oracle_mod):
    seqs = repeat_inputs.n_gapped(G=4, n=80_000, gaps=((10_000, 3000), (50_000, 1800)), shift=300, seed=19)
    check(gpu_lib, oracle_mod, seqs, 3, w=19, table_size=7)


@pytest.mark.parametrize("sp", [[0, 0, 0], [1000, 25_000, 7], [50_000, 0, 59_000]])
def test_start_points_plain(gpu_lib, oracle_mod, sp):
    seqs = oracle_mod.generate(3, 60_000, 0.02, 777)
    check(gpu_lib, oracle_mod, seqs, 3, start_points=sp)


@pytest.mark.parametrize("sp", [[1000, 25_000, 7], [3, 9_999, 10_001, 40_000]])
@pytest.mark.parametrize("layout", ["blocks", "slices"])
def test_start_points_with_restarts(gpu_lib, oracle_mod, sp, layout):
    seqs = repeat_inputs.n_gapped(G=len(sp), n=90_000, gaps=((2_000, 25_000), (60_000, 4_000)), shift=1_300,
                                  seed=31)
    check(gpu_lib, oracle_mod, seqs, 2, start_points=sp, layout=layout)


@pytest.mark.parametrize("sd", range(4))
def test_start_points_in_duplicate_runs(gpu_lib, oracle_mod, sd):
    rng = np.random.default_rng(200 + sd)
    seqs = tie_inputs.dup_block(seed=80 + sd)
    sp = [int(rng.integers(0, 30_000)), int(rng.integers(1, 50_000)), 0]
    check(gpu_lib, oracle_mod, seqs, 2 + sd % 3, start_points=sp)


def test_start_point_count_must_match(gpu_lib, oracle_mod):
    seqs = oracle_mod.generate(3, 20_000, 0.02, 9)
    with gpu_lib.ShardedMemHash([0] * 2, comm="local") as sh:
        sh.SetSeed(oracle_mod.get_seed(15))
        with pytest.raises(gpu_lib.MumsError):
            sh.FindMatchesFromPosition(seqs, [5, 7])
        assert sh.rank_status == [gpu_lib.MUMS_E_INVALID] * 2


@pytest.mark.parametrize("mode", ["local", "gather"])
@pytest.mark.parametrize("layout", ["blocks", "slices"])
def test_restart_memory_per_rank(gpu_lib, oracle_mod, monkeypatch, mode, layout):
    """The default plan allocates O(the rank's records) on every rank (its SML parts, 8 B per
    record, the live flags and their scan, 8 B per record, plus O(candidates) plan arrays); the
    gathered fallback allocates the whole stream's SMLs (8 B per seed-mer of every genome) on
    rank 0."""
    if mode == "gather":
        monkeypatch.setenv("MUMS_DEV_SHARD_RESTART", "gather")
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    info = []
    ref = check(gpu_lib, oracle_mod, seqs, 4, layout=layout, info=info)
    assert ref["restarts"] > 0
    L = gpu_lib.getSeedLength(oracle_mod.get_seed(15))
    N = sum(len(s) - L + 1 for s in seqs)
    world = len(info)
    if mode == "local":
        assert all(i["path"] == 1 for i in info), info
        for i in info:   # each rank: about 16 B x N / world (balanced key ranges) + small arrays
            assert i["bytes"] < 20 * N / world + (4 << 20), (i, N)
        assert info[0]["bytes"] < 8 * N, (info[0], N)
    else:
        assert all(i["path"] == 2 for i in info), info
        assert info[0]["bytes"] >= 8 * N, (info[0], N)
        assert all(i["bytes"] == 0 for i in info[1:]), info


def test_zz_path_counts(gpu_lib):
    """Report how many checks above planned locally and how many fell back (a key beyond a
    rank's neighbours): the fallback must stay the exception."""
    print("restart paths:", PATHS)
    if PATHS["local"] + PATHS["gather"] >= 20:
        assert PATHS["local"] >= PATHS["gather"], PATHS


# key ranges above one onesweep merge (2^30 records per rank: config 5 on 2 or 4 GPUs), forced
# small: mums_shard_merge merges the range in key chunks; the restart plans on the whole local
# stream, the live records are grouped chunk by chunk, and FindMatches takes every chunk's rows
@pytest.mark.parametrize("world,layout", [(2, "blocks"), (3, "blocks"), (2, "slices")])
def test_chunked_merge_restarts(gpu_lib, oracle_mod, monkeypatch, world, layout):
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    monkeypatch.setenv("MUMS_DEV_CHUNK_RECORDS", str(sum(len(s) for s in seqs) // (3 * world * 2)))
    ref = check(gpu_lib, oracle_mod, seqs, world, layout=layout)
    assert ref["restarts"] > 0


@pytest.mark.parametrize("sp", [[1000, 25_000, 7], [3, 9_999, 10_001, 40_000]])
def test_chunked_merge_start_points(gpu_lib, oracle_mod, monkeypatch, sp):
    seqs = repeat_inputs.n_gapped(G=len(sp), n=90_000, gaps=((2_000, 25_000), (60_000, 4_000)), shift=1_300,
                                  seed=31)
    # (the 25-kbp N runs put ~90 000 all-A seed-mers into one MSD bucket: a key chunk holds it)
    monkeypatch.setenv("MUMS_DEV_CHUNK_RECORDS", str(sum(len(s) for s in seqs) // 3))
    check(gpu_lib, oracle_mod, seqs, 2, start_points=sp)


@pytest.mark.parametrize("world", [2, 4])
def test_chunked_merge_findmatches(gpu_lib, oracle_mod, monkeypatch, world):
    seqs = oracle_mod.generate(4, 150_000, 0.02, 71)
    monkeypatch.setenv("MUMS_DEV_CHUNK_RECORDS", str(sum(len(s) for s in seqs) // (world * 4)))
    check(gpu_lib, oracle_mod, seqs, world, w=17)


# repeat tolerance (MemHash.cpp:139-162) over the ranks: every run of equal keys in std::sort
# order (mums_shard_tie_*), with and without restarts, one-pass and chunked merges
RTOL_CASES = {k: v for k, v in tie_inputs.CASES.items()
              if v[1].get("repeat_tol", 0) > 0 and v[1].get("enum_tol", 1) == 1}


@pytest.mark.parametrize("name", sorted(RTOL_CASES))
@pytest.mark.parametrize("world,layout", [(2, "blocks"), (3, "blocks"), (2, "slices")])
def test_repeat_tolerance(gpu_lib, oracle_mod, name, world, layout):
    gen, opts = RTOL_CASES[name]
    check(gpu_lib, oracle_mod, gen(), world, w=opts.get("w", 15), layout=layout, repeat_tol=opts["repeat_tol"])


@pytest.mark.parametrize("rtol", [1, 2])
@pytest.mark.parametrize("world,layout", [(2, "blocks"), (4, "blocks"), (3, "slices")])
def test_repeat_tolerance_with_restarts(gpu_lib, oracle_mod, rtol, world, layout):
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    ref = check(gpu_lib, oracle_mod, seqs, world, layout=layout, repeat_tol=rtol)
    assert ref["restarts"] > 0


@pytest.mark.parametrize("rtol", [1, 3])
def test_repeat_tolerance_chunked_merge(gpu_lib, oracle_mod, monkeypatch, rtol):
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    monkeypatch.setenv("MUMS_DEV_CHUNK_RECORDS", str(sum(len(s) for s in seqs) // 12))
    check(gpu_lib, oracle_mod, seqs, 2, repeat_tol=rtol)


# MatchFinder::LogProgress (MatchFinder.cpp:55-56, 296-309) over the ranks: the text of the
# whole merge, restated on rank 0 -- the single context's text (pinned to the oracle's
# literal SearchRange text by tests/test_gpu_progress.py)
@pytest.mark.parametrize("world,layout", [(2, "blocks"), (3, "blocks"), (2, "slices")])
@pytest.mark.parametrize("kind", ["plain", "n_gapped"])
def test_progress_text(gpu_lib, oracle_mod, world, layout, kind):
    if kind == "plain":
        seqs = oracle_mod.generate(3, 120_000, 0.02, 31)
    else:
        seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    seed = oracle_mod.get_seed(15)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        mh.LogProgress(True)
        ref_ml = mh.FindMatches(seqs)
        ref = mh.ProgressLog()
    assert ref.endswith("..") and "%" in ref
    with gpu_lib.ShardedMemHash([0] * (len(seqs) * 2 if layout == "slices" else world), comm="local",
                                layout=layout) as sh:
        sh.SetSeed(seed)
        sh.LogProgress(True)
        ml = sh.FindMatches(seqs)
        text = sh.ProgressLog()
    assert text == ref
    assert len(ml) == len(ref_ml)


def test_chunked_merge_gathered_plan_refused(gpu_lib, oracle_mod, monkeypatch):
    """A key-chunked merge whose local restart plan is undecidable (forced by the test hook; on
    real inputs a plan that needs keys beyond a rank's neighbours) ends every rank with
    MUMS_E_UNSUPPORTED and a message saying why, not the gathered plan's INVALID."""
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    monkeypatch.setenv("MUMS_DEV_CHUNK_RECORDS", str(sum(len(s) for s in seqs) // 12))
    monkeypatch.setenv("MUMS_DEV_SHARD_RESTART", "undecidable")
    with gpu_lib.ShardedMemHash([0] * 2, comm="local", table_size=40000) as sh:
        sh.SetSeed(oracle_mod.get_seed(15))
        with pytest.raises(gpu_lib.MumsError, match="key-chunked merge"):
            sh.FindMatches(seqs)
        assert sh.rank_status == [gpu_lib.MUMS_E_UNSUPPORTED] * 2


def test_undecidable_plan_falls_back_to_gathered(gpu_lib, oracle_mod, monkeypatch):
    """One-pass merges: an undecidable local plan falls back to the gathered plan, which gives
    the oracle's MatchList."""
    monkeypatch.setenv("MUMS_DEV_SHARD_RESTART", "undecidable")
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    info = []
    ref = check(gpu_lib, oracle_mod, seqs, 2, info=info)
    assert ref["restarts"] > 0 and all(i["path"] == 2 for i in info), info


# enumeration tolerance > 1 (MemHash.cpp:139-162, MatchFinder.cpp:342-393) over the ranks: each
# rank enumerates the groups of its key range, the copies in std::sort order (mums_shard_tie_*)
ETOL_CASES = {k: v for k, v in tie_inputs.CASES.items()
              if v[1].get("enum_tol", 1) > 1 and not v[1].get("cls") and v[1].get("w", 15) <= 21}


@pytest.mark.parametrize("name", sorted(ETOL_CASES))
@pytest.mark.parametrize("world,layout", [(2, "blocks"), (3, "slices")])
def test_enumeration_tolerance(gpu_lib, oracle_mod, name, world, layout):
    gen, o = ETOL_CASES[name]
    check(gpu_lib, oracle_mod, gen(), world, w=o.get("w", 15), layout=layout, repeat_tol=o.get("repeat_tol", 0),
          enum_tol=o["enum_tol"], start_points=o.get("start_points"))


@pytest.mark.parametrize("etol,rtol", [(2, 1), (3, 2), (8, 7), (12, 39)])
def test_enumeration_tolerance_repeats(gpu_lib, oracle_mod, etol, rtol):
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=40, tandem=False, seed=etol)
    check(gpu_lib, oracle_mod, seqs, 3, repeat_tol=rtol, enum_tol=etol)


@pytest.mark.parametrize("etol,rtol,w,layout", [(2, 1, 19, "blocks"), (3, 39, 19, "slices"), (12, 39, 21, "slices"),
                                                (2, 2, 20, "blocks")])
def test_enumeration_tolerance_ib33(gpu_lib, oracle_mod, monkeypatch, etol, rtol, w, layout):
    """Above 2^32 seed-mers (forced small: MUMS_DEV_SHARD_IB33) the ranks' merged records carry
    33-bit indices: the enumeration rows come from (full key, 64-bit index) pairs
    (groups.hip launch_rec_pairs33, mums_capi.hip shard_enum_rows)."""
    monkeypatch.setenv("MUMS_DEV_SHARD_IB33", "1")
    seqs = repeat_inputs.high_copy(G=3, n=60_000, copies=40, tandem=False, seed=etol + w)
    check(gpu_lib, oracle_mod, seqs, 3, w=w, layout=layout, repeat_tol=rtol, enum_tol=etol)


def test_enumeration_tolerance_with_restarts(gpu_lib, oracle_mod):
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    ref = check(gpu_lib, oracle_mod, seqs, 2, repeat_tol=1, enum_tol=2)
    assert ref["restarts"] > 0
