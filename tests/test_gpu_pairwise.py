"""GPU PairwiseMatchFinder (PairwiseMatchFinder.cpp:37-73; pairwise.hip) against the
oracle's restatement, bit for bit.  No reference fixture covers PairwiseMatchFinder:
parity rests on the oracle (its MemHash core is pinned by SURVEY Appendix C)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def gpu_pairwise(lm, seqs, seed, table_size=40000):
    with lm.PairwiseMatchFinder(0) as mh:
        mh.SetSeed(seed)
        mh.SetTableSize(table_size)
        ml = mh.FindMatches(seqs)
        return ml, mh.stats()


@pytest.mark.parametrize("G,n,p,w,gseed,T", [(3, 200000, 0.03, 15, 1, 40000), (4, 300000, 0.02, 15, 2, 40000),
                                            (2, 500000, 0.01, 19, 3, 40000), (5, 100000, 0.05, 11, 4, 40000),
                                            (3, 200000, 1.0, 9, 5, 40000), (4, 150000, 0.03, 17, 6, 7),
                                            (6, 80000, 0.02, 21, 7, 40000)])
def test_pairwise_vs_oracle(gpu_lib, oracle_mod, G, n, p, w, gseed, T):
    seqs = oracle_mod.generate(G, n, p, gseed)
    if G >= 3:   # a repeated region: genomes that occur twice drop out of the pairs
        seqs[1] = seqs[1][: n // 2] + seqs[0][1000:4000] * 2 + seqs[1][n // 2 + 6000:]
    seed = oracle_mod.get_seed(w)
    lengths, starts, st = oracle_mod.find_matches(seqs, seed, table_size=T, pairwise=True)
    ml, gst = gpu_pairwise(gpu_lib, seqs, seed, T)
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert gst["probes"] == st["probes"]
    assert ((ml.starts != 0).sum(axis=1) == 2).all()
