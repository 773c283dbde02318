"""GPU MemHash with enumeration tolerance > 1 (MemHash::EnumerateMatches, MemHash.cpp:139-162,
and the odometer of MatchFinder::EnumerateMatches, MatchFinder.cpp:342-393; pairwise.hip)
against the oracle's restatement, bit for bit.  Parity for enum_tol > 1 rests on the oracle
(no reference fixture covers it; its MemHash core is pinned by SURVEY Appendix C)."""
import pytest

from tests import repeat_inputs

pytestmark = pytest.mark.gpu


def with_repeats(oracle, G, n, p, gseed):
    seqs = oracle.generate(G, n, p, gseed)
    # copies of the same segments inside genomes: groups with several records per genome
    rep = seqs[0][5000:9000]
    return [s[: n // 3] + rep + s[n // 3 + 4000: 2 * n // 3] + rep + s[2 * n // 3 + 4000:] for s in seqs]


@pytest.mark.parametrize("G,n,p,w,rt,et,masked,mask", [(3, 200000, 0.02, 15, 1, 2, 0, 0), (3, 200000, 0.02, 15, 2, 3, 0, 0),
                                                      (4, 150000, 0.03, 15, 1, 2, 0, 0), (2, 300000, 0.01, 19, 3, 2, 0, 0),
                                                      (3, 200000, 0.02, 15, 1, 2, 1, 7), (3, 200000, 0.02, 15, 2, 2, 1, 0),
                                                      (4, 120000, 0.02, 17, 2, 8, 0, 0)])
def test_enumeration_tolerance_vs_oracle(gpu_lib, oracle_mod, G, n, p, w, rt, et, masked, mask):
    seqs = with_repeats(oracle_mod, G, n, p, 31 + G)
    seed = oracle_mod.get_seed(w)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, repeat_tol=rt, enum_tol=et, masked=bool(masked),
                                                   seq_mask=mask)
    cls = gpu_lib.MaskedMemHash if masked else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(seed)
        mh.SetRepeatTolerance(rt)
        mh.SetEnumerationTolerance(et)
        if masked:
            mh.SetMask(mask)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert st["probes"] == ost["probes"]
    assert st["collision_count"] == ost["collision_count"]


@pytest.mark.parametrize("et,rt,G,masked,mask", [(9, 8, 3, 0, 0), (12, 39, 3, 0, 0), (16, 15, 4, 0, 0),
                                                   (10, 39, 3, 1, 5), (11, 39, 3, 1, 0)])
def test_enumeration_tolerance_above_slot_bound(gpu_lib, oracle_mod, et, rt, G, masked, mask):
    """enum_tol above the slot kernels' 8 per-genome records (pairwise.hip en_*_walk_kernel):
    40 copies of one element per genome, so groups hold up to 40 records of a genome and the
    odometer runs up to et^G combinations per group."""
    seqs = repeat_inputs.high_copy(G=G, n=60_000, copies=40, tandem=False, seed=et)
    seed = oracle_mod.get_seed(15)
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, repeat_tol=rt, enum_tol=et, masked=bool(masked),
                                                   seq_mask=mask)
    cls = gpu_lib.MaskedMemHash if masked else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(seed)
        mh.SetRepeatTolerance(rt)
        mh.SetEnumerationTolerance(et)
        if masked:
            mh.SetMask(mask)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert st["probes"] == ost["probes"] > 0
    assert st["collision_count"] == ost["collision_count"]
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()


def test_enumeration_calls_above_row_stream_refused(gpu_lib, oracle_mod):
    """8 genomes with ~20 copies of one element each under enum_tol 20: a group's odometer has
    ~20^8 > 2^31 AddHashEntry calls, more than the row stream holds -- refused
    (MUMS_E_UNSUPPORTED, pairwise.hip en_rows32), never a wrapped row count."""
    seqs = repeat_inputs.high_copy(G=8, n=30_000, copies=20, tandem=False, seed=3)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(15))
        mh.SetRepeatTolerance(40)
        mh.SetEnumerationTolerance(20)
        with pytest.raises(gpu_lib.MumsError, match="2\\^31"):
            mh.FindMatches(seqs)
