"""GPU SeedOccurrenceList (SeedOccurrenceList.h:22-87), per-genome SortedMerList and the
MatchList filters (MatchList.h:636-664) against the oracle, bit for bit (float32 bits
for the frequencies)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(lm, seqs, seed, stage=None):
    mh = lm.MemHash(0)
    mh.SetSeed(seed)
    for s in seqs:
        mh.AddSequence(s)
    if stage is None:
        mh.CreateMatches()
    else:
        mh.FindStage(stage)
    return mh


@pytest.mark.parametrize("G,n,p,w,gseed", [(3, 200000, 0.02, 15, 1), (2, 50000, 1.0, 7, 2), (2, 300000, 0.01, 19, 3),
                                          (2, 100000, 1.0, 5, 4)])
def test_seed_occurrence_vs_oracle(gpu_lib, oracle_mod, G, n, p, w, gseed):
    seqs = oracle_mod.generate(G, n, p, gseed)
    seqs[1] = seqs[1][: n // 2] + seqs[0][:5000] * 3          # repeats -> frequencies > 1
    seed = oracle_mod.get_seed(w)
    with _run(gpu_lib, seqs, seed, gpu_lib.STAGE_SEEDS) as mh:
        for g, s in enumerate(seqs):
            ref = oracle_mod.seed_occurrence(s, seed)
            got = mh.SeedOccurrence(g, len(s))
            assert (got.view(np.uint32) == ref.view(np.uint32)).all()
            sml = mh.SortedMerList(g, max(len(s) - oracle_mod.lib().oracle_seed_length(seed) + 1, 0))
            assert (sml == oracle_mod.build_sml(s, seed)).all()


def test_seed_occurrence_short_and_tiny(gpu_lib, oracle_mod):
    seed = oracle_mod.get_seed(15)
    seqs = [b"ACGTACGTAC", b"A", b"ACGTTGCA" * 3 + b"ACG", oracle_mod.generate(1, 5000, 1.0, 9)[0]]
    with _run(gpu_lib, seqs, seed, gpu_lib.STAGE_SEEDS) as mh:
        for g, s in enumerate(seqs):
            ref = oracle_mod.seed_occurrence(s, seed)
            assert (mh.SeedOccurrence(g, len(s)).view(np.uint32) == ref.view(np.uint32)).all()


def test_match_filters(gpu_lib, oracle_mod):
    seqs = oracle_mod.generate(4, 300000, 0.03, 11)
    seed = oracle_mod.get_seed(15)
    lengths, starts, _ = oracle_mod.find_matches(seqs, seed)
    mult = (starts != 0).sum(axis=1)
    with _run(gpu_lib, seqs, seed) as mh:
        ml = mh.GetMatchList()
        assert (ml.lengths == lengths).all()
        mh.MultiplicityFilter(3)
        f = mh.GetMatchList()
        keep = mult == 3
        assert 0 < len(f) < len(ml)
        assert (f.lengths == lengths[keep]).all() and (f.starts == starts[keep]).all()
        mh.LengthFilter(40)
        f2 = mh.GetMatchList()
        keep2 = keep & (lengths >= 40)
        assert (f2.lengths == lengths[keep2]).all() and (f2.starts == starts[keep2]).all()
        mh.LengthFilter(10 ** 9)
        assert len(mh.GetMatchList()) == 0
