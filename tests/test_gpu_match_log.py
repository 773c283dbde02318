"""MemHash::SetMatchLog (MemHash.h:149; MemHash.cpp:238-241): the entries the log stream
receives, in insertion (AddHashEntry call) order, = the oracle's inserts in its call order,
on every replay path (per-bucket rounds, the whole-bucket fast path, the big-bucket rank
counts with suspicious probes and their closed-form rounds, forced onto small buckets by
MUMS_DEV_BIG_BUCKET / MUMS_DEV_GRID_SLOW)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("G,n,w,p,table_size,big", [(3, 200_000, 15, 0.03, 40000, None), (4, 1_000_000, 15, 0.01, 40000, None),
                                                   (4, 1_000_000, 15, 0.01, 40000, "8"), (5, 300_000, 13, 0.02, 7, None),
                                                   (4, 500_000, 15, 1.0, 40000, None), (3, 400_000, 11, 0.05, 1, "8"),
                                                   (4, 1_000_000, 15, 0.01, 40000, "8+closed")])
def test_match_log_order(gpu_lib, oracle_mod, monkeypatch, G, n, w, p, table_size, big):
    if big:
        monkeypatch.setenv("MUMS_DEV_BIG_BUCKET", big.split("+")[0])
        if big.endswith("+closed"):   # the closed-form big-bucket rounds (bigq_*)
            monkeypatch.setenv("MUMS_DEV_GRID_SLOW", "0")
    seqs = oracle_mod.generate(G, n, p, 31 + G + w)
    seed = oracle_mod.get_seed(w)
    _, _, st = oracle_mod.find_matches(seqs, seed, table_size=table_size)
    ref_len, ref_s = st["match_log"]
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        mh.SetTableSize(table_size)
        mh.SetMatchLog(True)
        mh.FindMatches(seqs)
        log = mh.MatchLog()
    assert len(log) == len(ref_len) == st["mem_count"]
    assert np.array_equal(log.lengths, ref_len) and np.array_equal(log.starts, ref_s)


def test_match_log_off_refuses(gpu_lib, oracle_mod):
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(15))
        mh.FindMatches(oracle_mod.generate(2, 100_000, 0.02, 3))
        with pytest.raises(gpu_lib.MumsError):
            mh.MatchLog()
