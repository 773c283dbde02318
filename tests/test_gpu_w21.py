"""Seed weights 20-21 on one context.  getSeed(21) is getDefaultSeedWeight's choice for genomes
above ~1.07 Gbp (SeedMasks.h:389-401 via MatchList.h:351-357), so mauveAligner uses it on
mammalian assemblies.  Its 43-bit keys leave 11 bits outside the packed record: the keys pass
scatters by the top 8 bits and keeps the next 2w+1-40 bits in a side byte, and msd_split
(msdsplit.hip) partitions the 256 buckets into the 2^(2w+1-32) buckets the sort runs in.
GPU against the oracle bit for bit, and split against the one-level 2^B-digit scatter
(MUMS_DEV_NO_SPLIT) on larger inputs."""
import os

import numpy as np
import pytest

from tests import repeat_inputs

pytestmark = pytest.mark.gpu


def gpu_find(lm, seqs, seed, cls="MemHash", mask=0, **kw):
    with getattr(lm, cls)(0) as mh:
        mh.SetSeed(seed)
        if "table_size" in kw:
            mh.SetTableSize(kw["table_size"])
        mh.SetRepeatTolerance(kw.get("repeat_tol", 0))
        mh.SetEnumerationTolerance(kw.get("enum_tol", 1))
        if cls == "MaskedMemHash":
            mh.SetMask(mask)
        ml = mh.FindMatches(seqs)
        return ml, mh.stats()


def check(lm, oracle_mod, seqs, seed, cls="MemHash", mask=0, **kw):
    ml, st = gpu_find(lm, seqs, seed, cls, mask, **kw)
    ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, seed, masked=cls == "MaskedMemHash", seq_mask=mask, **kw)
    assert len(ml) == len(ref_len)
    assert (ml.lengths == ref_len).all()
    assert (ml.starts == ref_starts).all()
    assert st["collision_count"] == ref["collision_count"]
    assert st["mem_count"] == ref["mem_count"]
    return st, ref


@pytest.mark.parametrize("w,rank", [(21, 0), (21, 2), (20, 0), (20, 1), (20, 2)])
def test_w2x_patterns(gpu_lib, oracle_mod, w, rank):
    seqs = oracle_mod.generate(3, 150_000, 0.01, 300 + w + rank)
    check(gpu_lib, oracle_mod, seqs, oracle_mod.get_seed(w, rank))


@pytest.mark.parametrize("G,n,p,cls,mask,kw", [
    (5, 120_000, 0.01, "MemHash", 0, {}),
    (2, 300_000, 1.0, "MemHash", 0, {}),                       # unrelated: single-copy keys only
    (4, 150_000, 0.02, "MaskedMemHash", 0b1011, {}),
    (4, 150_000, 0.02, "MemHash", 0, {"table_size": 7}),
    (3, 150_000, 0.05, "MemHash", 0, {"repeat_tol": 1}),      # SML std::sort tie order
    (9, 40_000, 0.02, "MemHash", 0, {}),                       # MG=16 kernels
])
def test_w21_shapes(gpu_lib, oracle_mod, G, n, p, cls, mask, kw):
    seqs = oracle_mod.generate(G, n, p, 4000 + G)
    check(gpu_lib, oracle_mod, seqs, oracle_mod.get_seed(21), cls, mask, **kw)


def test_w21_seed_keys_and_sml(gpu_lib, oracle_mod):
    seqs = oracle_mod.generate(3, 80_000, 0.03, 21)
    seed = oracle_mod.get_seed(21)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        for s in seqs:
            mh.AddSequence(s)
        mh.FindStage(gpu_lib.STAGE_SEEDS)
        for g, s in enumerate(seqs):
            ref = oracle_mod.seed_keys(s, seed)
            assert (mh.SeedKeys(g, len(ref)) == ref).all()
            assert (mh.SortedMerList(g, len(ref)) == oracle_mod.build_sml(s, seed)).all()


@pytest.mark.parametrize("cls,mask", [("MemHash", 0), ("MaskedMemHash", 5)])
def test_w21_restart_n_gapped(gpu_lib, oracle_mod, cls, mask):
    """N runs give one all-A key group per gap (MER_REPEAT_LIMIT restarts, MatchFinder.cpp:253-277)."""
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 2500)), shift=300, seed=3)
    st, ref = check(gpu_lib, oracle_mod, seqs, oracle_mod.get_seed(21), cls, mask)
    assert ref["restarts"] > 0 and st["restarts"] == ref["restarts"]


def test_w21_split_equals_one_level_scatter(gpu_lib, oracle_mod, monkeypatch):
    """8 x 2 Mbp related: the split layout gives the same stream as the 2^11-digit scatter, so
    the MatchList and every counter agree."""
    seqs = oracle_mod.generate(8, 2_000_000, 0.01, 99)
    seed = oracle_mod.get_seed(21)
    ml_a, st_a = gpu_find(gpu_lib, seqs, seed)
    monkeypatch.setenv("MUMS_DEV_NO_SPLIT", "1")
    ml_b, st_b = gpu_find(gpu_lib, seqs, seed)
    assert len(ml_a) == len(ml_b) > 0
    assert (ml_a.lengths == ml_b.lengths).all() and (ml_a.starts == ml_b.starts).all()
    for k in ("collision_count", "mem_count", "probes", "groups", "chains"):
        assert st_a[k] == st_b[k], k


def test_default_weight_of_mammalian_genomes(gpu_lib):
    assert gpu_lib.getDefaultSeedWeight(3_000_000_000) == 21
    assert gpu_lib.getDefaultSeedWeight(1_100_000_000) == 21
    assert gpu_lib.getSeed(21) == 0x7ddaddf
