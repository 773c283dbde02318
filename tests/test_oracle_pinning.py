"""The CPU oracle against the reference's own known answers.

Every case regenerates the Appendix-C synthetic input (std::mt19937_64 seed 12345),
runs the oracle MemHash / MaskedMemHash and compares the md5 of the MatchList
text with the md5 the reference produced.  This pins the oracle that the GPU
parity tests use as their checker.
"""
import hashlib
import json
import os

import pytest

from conftest import GOLDEN

CASES = json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["cases"]


def _run(oracle, c, **kw):
    seqs = oracle.generate(c["G"], c["n"], c["p"], 12345)
    masked = c["mode"] == "MaskedMemHash"
    return oracle.find_matches(seqs, oracle.get_seed(c["w"]), masked=masked, seq_mask=c.get("mask", 0), **kw)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}_{c['mode']}")
def test_oracle_matches_reference_md5(oracle_mod, case):
    lengths, starts, st = _run(oracle_mod, case)
    txt = oracle_mod.match_text(lengths, starts)
    assert len(lengths) == case["matches"]
    assert hashlib.md5(txt.encode()).hexdigest() == case["md5"]
    if "collisions" in case:
        assert st["collision_count"] == case["collisions"]
    if "first_line" in case:
        assert txt.split("\n", 1)[0] == case["first_line"]
    if "duplicate_pair" in case:
        lines = txt.splitlines()
        dup = [i for i in range(len(lines) - 1) if lines[i] == lines[i + 1]]
        assert len(dup) == 1 and lines[dup[0]] == case["duplicate_pair"]
    # no group reached MER_REPEAT_LIMIT, so the restart path (MatchFinder.cpp:253-277) is not exercised
    assert st["max_group"] <= 1000


@pytest.mark.parametrize("name", ["c1_related.txt", "c1_iid.txt", "g3_200k_p003.txt"])
def test_golden_fixture_files_match_md5(name):
    txt = open(os.path.join(GOLDEN, name)).read()
    md5 = hashlib.md5(txt.encode()).hexdigest()
    assert md5 in {c["md5"] for c in CASES}


@pytest.mark.parametrize("G,n,p", [(3, 200000, 0.03), (2, 1000000, 0.01), (3, 300000, 0.05)])
def test_extension_insensitive_to_gnseqi_end(oracle_mod, G, n, p):
    """GNSEQI_END (UINT64_MAX -> maxlen -1, no L-jumps) changes speed, not results."""
    seqs = oracle_mod.generate(G, n, p, 12345)
    a = oracle_mod.find_matches(seqs, oracle_mod.get_seed(15), gnseqi_end_neg1=False)
    b = oracle_mod.find_matches(seqs, oracle_mod.get_seed(15), gnseqi_end_neg1=True)
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all()


PCOMPAT = json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["parallel_compat"]


@pytest.mark.parametrize("case", PCOMPAT, ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}_ParallelMemHash")
def test_oracle_parallel_compat_matches_reference_md5(oracle_mod, case):
    """ParallelMemHash (patched) known answer: the oracle's restatement of
    ParallelMemHash::FindMatches (chunking by GetBreakpoint, per-chunk SearchRange, MergeTable)
    reproduces the reference's 15 893-match MatchList byte for byte."""
    seqs = oracle_mod.generate(case["G"], case["n"], case["p"], 12345)
    lengths, starts, st = oracle_mod.find_matches(seqs, oracle_mod.get_seed(case["w"]), parallel_compat=True,
                                                  chunk_size=case["chunk_size"])
    txt = oracle_mod.match_text(lengths, starts)
    assert st["chunks"] == case["chunks"]
    assert len(lengths) == case["matches"]
    assert hashlib.md5(txt.encode()).hexdigest() == case["md5"]
    assert txt.count("\n") == len(set(txt.splitlines()))   # MergeTable collapsed the serial duplicate


# (G, n, p, w, chunk_size, generator seed): many chunks on small inputs
COMPAT_SMALL = [(2, 200000, 0.01, 15, 5000, 1), (3, 300000, 0.03, 15, 3000, 2), (4, 200000, 0.01, 15, 2000, 3),
                (3, 500000, 0.05, 15, 7000, 4), (3, 200000, 1.0, 11, 1003, 6), (3, 200000, 0.01, 12, 999, 8)]


@pytest.mark.parametrize("G,n,p,w,chunk,gseed", COMPAT_SMALL)
def test_parallel_compat_deferred_merge_equivalent(oracle_mod, G, n, p, w, chunk, gseed):
    """The GPU reproduces MergeTable once, after all chunks (compat.hip); the literal
    restatement merges after every chunk.  Both give the same MatchList (which differs from
    serial MemHash's at the chunk boundaries)."""
    seqs = oracle_mod.generate(G, n, p, gseed)
    seed = oracle_mod.get_seed(w)
    a = oracle_mod.find_matches(seqs, seed, parallel_compat=1, chunk_size=chunk)
    b = oracle_mod.find_matches(seqs, seed, parallel_compat=2, chunk_size=chunk)
    ta, tb = (oracle_mod.match_text(x[0], x[1]) for x in (a, b))
    assert ta == tb
    assert a[2]["chunks"] > 10


@pytest.mark.parametrize("n,p,gseed", [(1000000, 0.01, 12345), (1000000, 1.0, 12345), (300000, 0.05, 3)])
def test_pairwise_equals_memhash_for_two_genomes(oracle_mod, n, p, gseed):
    """PairwiseMatchFinder (PairwiseMatchFinder.cpp:37-73) with two genomes hashes exactly the
    probes MemHash does (both single-copy <=> MemHash's repeat_tol 0 acceptance), so its
    MatchList equals MemHash's, which is pinned to the reference for the first two cases."""
    seqs = oracle_mod.generate(2, n, p, gseed)
    seed = oracle_mod.get_seed(15)
    a = oracle_mod.find_matches(seqs, seed, pairwise=True)
    b = oracle_mod.find_matches(seqs, seed)
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all() and a[2]["probes"] == b[2]["probes"]
