"""The oracle's ParallelMemHash LogProgress / SetMatchLog restatement (one OpenMP thread,
SURVEY.md B.3), pinned by identities with the serial MemHash oracle: with a single chunk the
progress text is MemHash's, and the match log is MemHash's inserts followed by MergeTable's
re-adds of the whole table, i.e. the final MatchList in bucket order.  With many chunks every
final entry appears exactly once after its chunk's thread-table insert."""
import numpy as np
import pytest


@pytest.mark.parametrize("G,n,p,w", [(3, 150_000, 0.02, 13), (2, 200_000, 1.0, 11), (4, 120_000, 0.01, 15)])
def test_one_chunk_is_memhash_then_merge(oracle_mod, G, n, p, w):
    seqs = oracle_mod.generate(G, n, p, 5 + G)
    seed = oracle_mod.get_seed(w)
    lc, sc, xc = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=10 * n)
    lm, sm, xm = oracle_mod.find_matches(seqs, seed)
    assert xc["chunks"] == 1
    assert xc["progress"] == xm["progress"] and xm["progress"]
    k = len(xm["match_log"][0])
    assert len(xc["match_log"][0]) == k + len(lc)
    assert np.array_equal(xc["match_log"][0][:k], xm["match_log"][0])
    assert np.array_equal(xc["match_log"][1][:k], xm["match_log"][1])
    assert np.array_equal(xc["match_log"][0][k:], lc) and np.array_equal(xc["match_log"][1][k:], sc)


def test_many_chunks_log_covers_the_list(oracle_mod):
    seqs = oracle_mod.generate(3, 300_000, 0.03, 2)
    seed = oracle_mod.get_seed(15)
    lc, sc, xc = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=3000)
    assert xc["chunks"] > 50
    ll, ls = xc["match_log"]
    rows = {(int(a), *map(int, b)) for a, b in zip(ll, ls)}
    assert all((int(a), *map(int, b)) in rows for a, b in zip(lc, sc))
    assert len(ll) >= 2 * len(lc)
    # the text counts every chunk's buffers: the percentages only grow, one line per ten
    pct = [int(t) for t in xc["progress"].replace("\n", "").split("%..") if t]
    assert pct == sorted(pct) and pct[0] == 0


@pytest.mark.parametrize("G,n,p,w,chunk,gseed,ranks", [(3, 300_000, 0.03, 15, 3000, 2, 3), (4, 200_000, 0.01, 15, 2000, 3, 8),
                                                       (3, 200_000, 1.0, 11, 1003, 6, 4), (5, 300_000, 0.02, 17, 4000, 9, 2)])
def test_chunk_range_ranks_model(oracle_mod, G, n, p, w, chunk, gseed, ranks):
    """The oracle's model of chunk-parallel ranks (parallel_compat = 16 + ranks: each rank
    searches a contiguous chunk range into tables of its own, never synced, and the ranks'
    global tables are re-added rank after rank at the end) gives the one-thread reference's
    MatchList -- the schedule independence SURVEY.md §8 row A13 reports for 1/4/8 OpenMP
    threads, the basis of a multi-GPU compat mode."""
    seqs = oracle_mod.generate(G, n, p, gseed)
    seed = oracle_mod.get_seed(w)
    l1, s1, x1 = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
    lr, sr, xr = oracle_mod.find_matches(seqs, seed, parallel_compat=16 + ranks, chunk_size=chunk)
    assert x1["chunks"] == xr["chunks"] > ranks
    assert np.array_equal(l1, lr) and np.array_equal(s1, sr)
