"""The OpenMP CPU path of the oracle (oracle_find_matches_omp: per-genome SMLs in parallel,
merge split by key range, hash buckets replayed in parallel -- the bench's CPU baseline on
the host cores) equals the serial restatement bit for bit."""
import numpy as np
import pytest

from tests import repeat_inputs


def same(a, b):
    la, sa, ta = a
    lb, sb, tb = b
    assert len(la) == len(lb)
    assert (la == lb).all() and (sa == sb).all()
    for k in ("mem_count", "collision_count", "probes", "seedmers"):
        assert ta[k] == tb[k], k


@pytest.mark.parametrize("G,n,w,p,threads", [(2, 300_000, 15, 0.01, 4), (3, 200_000, 15, 0.03, 8),
                                              (4, 400_000, 15, 1.0, 3), (5, 250_000, 19, 0.02, 8),
                                              (3, 200_000, 11, 0.05, 2)])
def test_omp_equals_serial(oracle_mod, G, n, w, p, threads):
    seqs = oracle_mod.generate(G, n, p, 4242)
    seed = oracle_mod.get_seed(w)
    same(oracle_mod.find_matches(seqs, seed, omp_threads=threads), oracle_mod.find_matches(seqs, seed))


def test_omp_masked_and_tolerances(oracle_mod):
    seqs = oracle_mod.generate(3, 200_000, 0.02, 99)
    seed = oracle_mod.get_seed(15)
    for kw in (dict(masked=True, seq_mask=7), dict(masked=True, seq_mask=5), dict(repeat_tol=1, enum_tol=2),
               dict(pairwise=True), dict(table_size=7)):
        same(oracle_mod.find_matches(seqs, seed, omp_threads=6, **kw), oracle_mod.find_matches(seqs, seed, **kw))


def test_omp_seeds_only_probe_log(oracle_mod):
    seqs = oracle_mod.generate(4, 300_000, 0.01, 7)
    seed = oracle_mod.get_seed(15)
    a = oracle_mod.seed_probes(seqs, seed, omp_threads=5)
    b = oracle_mod.seed_probes(seqs, seed)
    assert len(a[0]) > 1000
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert a[2]["probes"] == b[2]["probes"] and a[2]["seedmers"] == b[2]["seedmers"]


def test_omp_restarting_merge_falls_back(oracle_mod):
    seqs = repeat_inputs.n_gapped(G=3, n=60_000, gaps=((20_000, 3000),), seed=3)
    seed = oracle_mod.get_seed(15)
    a = oracle_mod.find_matches(seqs, seed, omp_threads=4)
    b = oracle_mod.find_matches(seqs, seed)
    same(a, b)
    assert a[2]["restarts"] == b[2]["restarts"] >= 1
