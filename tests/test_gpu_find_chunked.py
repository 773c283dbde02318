"""FindMatches in slices (find_rows_chunked: BASELINE config 5 has 2.5e9 AddHashEntry
calls, more than the one-pass replay's per-probe arrays hold): chains labelled per slice
of the probes and merged by entry content, then the replay over chunks of the bucket
order.  Forced onto small inputs with MUMS_DEV_FIND_CHUNK (probes per slice) and checked
bit for bit against the oracle, the Appendix-C known answers and the one-pass path
(same merged chain count, same match log)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

CASES = [c for c in json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["cases"] if c["mode"] != "ParallelMemHash"]


@pytest.fixture
def find_chunk(monkeypatch):
    def _set(n):
        monkeypatch.setenv("MUMS_DEV_FIND_CHUNK", str(n))
    return _set


def run(gpu_lib, seqs, seed, masked=0, table_size=None, log=False):
    cls = gpu_lib.MaskedMemHash if masked else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(seed)
        if masked:
            mh.SetMask(masked)
        if table_size:
            mh.SetTableSize(table_size)
        if log:
            mh.SetMatchLog(True)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
        lg = mh.MatchLog() if log else None
    return ml, st, lg


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}_{c['mode']}")
def test_find_chunked_known_answers(gpu_lib, oracle_mod, case, find_chunk):
    seqs = oracle_mod.generate(case["G"], case["n"], case["p"], 12345)
    find_chunk(1_000_003)
    ml, st, _ = run(gpu_lib, seqs, oracle_mod.get_seed(case["w"]),
                    masked=case.get("mask", 0) if case["mode"] == "MaskedMemHash" else 0)
    if st["probes"] <= 1_000_003:
        pytest.skip("fewer probes than one slice")
    assert len(ml) == case["matches"]
    assert hashlib.md5(ml.text().encode()).hexdigest() == case["md5"]
    if "collisions" in case:
        assert st["collision_count"] == case["collisions"]


@pytest.mark.parametrize("G,n,p,w,chunk,masked,table_size", [
    (2, 400_000, 0.01, 15, 50_000, 0, None),
    (3, 300_000, 0.02, 13, 7_919, 0, None),
    (4, 200_000, 0.03, 15, 100_000, 0, 7),       # 7 buckets: every bucket on the big paths
    (5, 100_000, 0.05, 11, 33_333, 0, 1),        # one bucket
    (3, 300_000, 0.02, 15, 20_000, 7, None),     # MaskedMemHash
    (6, 150_000, 0.01, 15, 64, 0, None),         # thousands of slices
    (3, 200_000, 1.0, 11, 5_000, 0, None),       # unrelated: short chains, few duplicates
])
def test_find_chunked_vs_oracle(gpu_lib, oracle_mod, find_chunk, G, n, p, w, chunk, masked, table_size):
    seqs = oracle_mod.generate(G, n, p, 31 + G + w)
    seed = oracle_mod.get_seed(w)
    kw = dict(table_size=table_size) if table_size else {}
    lengths, starts, ost = oracle_mod.find_matches(seqs, seed, masked=bool(masked), seq_mask=masked, **kw)
    _, one, lg1 = run(gpu_lib, seqs, seed, masked, table_size, log=True)
    find_chunk(chunk)
    ml, st, lg = run(gpu_lib, seqs, seed, masked, table_size, log=True)
    assert st["probes"] > chunk
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert st["collision_count"] == ost["collision_count"] and st["mem_count"] == ost["mem_count"]
    # the merged chains are the one-pass path's chains; the inserts come in the same order
    assert st["chains"] == one["chains"]
    assert np.array_equal(lg.lengths, lg1.lengths) and np.array_equal(lg.starts, lg1.starts)


def test_find_chunked_reuse(gpu_lib, oracle_mod, find_chunk):
    """One context: one-pass, sliced, one-pass again (buffers released / regrown)."""
    seqs = oracle_mod.generate(3, 200_000, 0.02, 4)
    seed = oracle_mod.get_seed(13)
    lengths, starts, _ = oracle_mod.find_matches(seqs, seed)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        for s in seqs:
            mh.AddSequence(s)
        for chunk in (None, 10_000, None, 123_457):
            if chunk:
                os.environ["MUMS_DEV_FIND_CHUNK"] = str(chunk)
            try:
                mh.CreateMatches()
            finally:
                os.environ.pop("MUMS_DEV_FIND_CHUNK", None)
            ml = mh.GetMatchList()
            assert (ml.lengths == lengths).all() and (ml.starts == starts).all()


PCOMPAT = json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["parallel_compat"]


@pytest.mark.parametrize("chunk", [1_000_003, 77_777])
def test_find_chunked_parallel_compat(gpu_lib, oracle_mod, find_chunk, chunk):
    """ParallelMemHash compat through the sliced FindMatches (its chunk-major stream, 64-bit
    rows per slice, MergeTable on the merged chain pool): the reference md5 fa9dea6f... of
    4 x 10 Mbp, and a small shape against the oracle."""
    case = PCOMPAT[0]
    seqs = oracle_mod.generate(case["G"], case["n"], case["p"], 12345)
    find_chunk(chunk)
    with gpu_lib.ParallelMemHash(0, case["chunk_size"]) as mh:
        mh.SetSeed(oracle_mod.get_seed(case["w"]))
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert st["probes"] > chunk
    assert st["chunks"] == case["chunks"] and len(ml) == case["matches"]
    assert hashlib.md5(ml.text().encode()).hexdigest() == case["md5"]
    seqs = oracle_mod.generate(3, 300_000, 0.03, 2)
    seed = oracle_mod.get_seed(15)
    lengths, starts, _ = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=3000)
    find_chunk(max(1, chunk // 100))
    with gpu_lib.ParallelMemHash(0, 3000) as mh:
        mh.SetSeed(seed)
        ml = mh.FindMatches(seqs)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
