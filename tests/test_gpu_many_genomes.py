"""More than 32 genomes per context (up to 64, MaskedMemHash's 64-bit match number,
MaskedMemHash.cpp:51-58): MemHash and MaskedMemHash FindMatches on 33-64 related genomes
against the oracle, incl. the 64-bit masks (all genomes, all but one), the sliced
FindMatches, and the paths with their own kernels (PairwiseMatchFinder, enumeration
tolerance > 1: 64-bit genome masks above 32 genomes; ParallelMemHash compat: 64-genome
MergeTable)."""
import pytest

pytestmark = pytest.mark.gpu


def gpu_find(gpu_lib, seqs, seed, mask=None, table_size=None):
    cls = gpu_lib.MaskedMemHash if mask is not None else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(seed)
        if mask is not None:
            mh.SetMask(mask)
        if table_size:
            mh.SetTableSize(table_size)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    return ml, st


def check(ml, st, ref):
    lengths, starts, ost = ref
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert st["probes"] == ost["probes"] and st["mem_count"] == ost["mem_count"]
    assert st["collision_count"] == ost["collision_count"]


@pytest.mark.parametrize("G,n,p,w,table_size", [(33, 20000, 0.01, 13, None), (40, 30000, 0.005, 15, None),
                                                (64, 20000, 0.003, 13, None), (48, 20000, 0.01, 11, 97)])
def test_memhash_many_genomes(gpu_lib, oracle_mod, G, n, p, w, table_size):
    seqs = oracle_mod.generate(G, n, p, 700 + G)
    seed = oracle_mod.get_seed(w)
    kw = dict(table_size=table_size) if table_size else {}
    ref = oracle_mod.find_matches(seqs, seed, **kw)
    assert len(ref[0]) > 0
    ml, st = gpu_find(gpu_lib, seqs, seed, table_size=table_size)
    check(ml, st, ref)


@pytest.mark.parametrize("G", [36, 64])
@pytest.mark.parametrize("which", ["all", "all_but_one"])
def test_masked_memhash_64bit_masks(gpu_lib, oracle_mod, G, which):
    seqs = oracle_mod.generate(G, 20000, 0.003, 900 + G)
    seed = oracle_mod.get_seed(13)
    full = (1 << G) - 1
    mask = {"all": full, "all_but_one": full & ~(1 << (G - 1 - 5))}[which]   # genome 0 = top bit
    ref = oracle_mod.find_matches(seqs, seed, masked=True, seq_mask=mask)
    assert len(ref[0]) > 0
    ml, st = gpu_find(gpu_lib, seqs, seed, mask=mask)
    check(ml, st, ref)


def test_many_genomes_sliced_findmatches(gpu_lib, oracle_mod, monkeypatch):
    seqs = oracle_mod.generate(40, 20000, 0.01, 5)
    seed = oracle_mod.get_seed(13)
    ref = oracle_mod.find_matches(seqs, seed)
    monkeypatch.setenv("MUMS_DEV_FIND_CHUNK", "3000")
    ml, st = gpu_find(gpu_lib, seqs, seed)
    assert st["probes"] > 3000
    check(ml, st, ref)


@pytest.mark.parametrize("G,n,p,w,kind", [(40, 3000, 0.01, 13, "pairwise"), (64, 1500, 0.005, 11, "pairwise"),
                                           (36, 20000, 0.01, 13, "enum2"), (36, 20000, 1.0, 13, "enum3_rep1"),
                                           (40, 30000, 0.01, 13, "compat")])
def test_more_than_32_genomes_other_finders(gpu_lib, oracle_mod, G, n, p, w, kind):
    seqs = oracle_mod.generate(G, n, p, 1300 + G)
    seed = oracle_mod.get_seed(w)
    kw, cls, setup = {}, gpu_lib.MemHash, {}
    if kind == "pairwise":
        kw, cls = dict(pairwise=True), gpu_lib.PairwiseMatchFinder
    elif kind == "enum2":
        kw = setup = dict(enum_tol=2)
    elif kind == "enum3_rep1":
        kw = setup = dict(enum_tol=3, repeat_tol=1)
    else:
        kw, cls = dict(parallel_compat=True, chunk_size=20000), None
    ref = oracle_mod.find_matches(seqs, seed, **kw)
    assert len(ref[0]) > 0
    mh = gpu_lib.ParallelMemHash(0, chunk_size=20000) if cls is None else cls(0)
    with mh:
        mh.SetSeed(seed)
        if "enum_tol" in setup:
            mh.SetEnumerationTolerance(setup["enum_tol"])
        if "repeat_tol" in setup:
            mh.SetRepeatTolerance(setup["repeat_tol"])
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    lengths, starts, ost = ref
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert st["mem_count"] == ost["mem_count"]
    if kind != "compat":   # ParallelMemHash's collision counter is bumped by every OpenMP thread unguarded
        assert st["collision_count"] == ost["collision_count"]   # (MemHash.cpp:218 via ParallelMemHash.cpp:114,126): not a defined output
