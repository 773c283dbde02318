"""More than 32 genomes per context (up to 64, MaskedMemHash's 64-bit match number,
MaskedMemHash.cpp:51-58): MemHash and MaskedMemHash FindMatches on 33-64 related genomes
against the oracle, incl. the 64-bit masks (all genomes, all but one), the sliced
FindMatches, and the refusal of the paths that stay at 32 (PairwiseMatchFinder,
enumeration tolerance > 1, ParallelMemHash compat)."""
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


def test_more_than_32_genomes_refused_on_32_genome_paths(gpu_lib, oracle_mod):
    seqs = oracle_mod.generate(33, 5000, 0.01, 3)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(11))
        mh.SetEnumerationTolerance(2)
        with pytest.raises(gpu_lib.MumsError):
            mh.FindMatches(seqs)
