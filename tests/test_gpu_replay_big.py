"""The big-bucket replay (replay_big_kernel: chain-rank counts + exact lower_bound for the
suspicious probes; the closed-form rounds of bigq_* for buckets with many suspicious probes)
forced onto small buckets (MUMS_DEV_BIG_BUCKET, MUMS_DEV_GRID_SLOW), bit-exact against the
reference known answers (incl. the 4 x 10 Mbp related case whose main-diagonal bucket holds
the duplicated entry of SURVEY.md §0.4) and the oracle on varied shapes."""
import hashlib
import json
import os

import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

CASES = [c for c in json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["cases"] if c["mode"] != "ParallelMemHash"]


@pytest.fixture(params=["rank_counts", "closed_form"])
def force_big(monkeypatch, request):
    monkeypatch.setenv("MUMS_DEV_BIG_BUCKET", "8")
    if request.param == "closed_form":   # every untied big bucket through bigq_* (replay.hip)
        monkeypatch.setenv("MUMS_DEV_GRID_SLOW", "0")


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}_{c['mode']}")
def test_big_bucket_replay_known_answers(gpu_lib, oracle_mod, case, force_big):
    seqs = oracle_mod.generate(case["G"], case["n"], case["p"], 12345)
    cls = gpu_lib.MaskedMemHash if case["mode"] == "MaskedMemHash" else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(case["w"]))
        if case["mode"] == "MaskedMemHash":
            mh.SetMask(case.get("mask", 0))
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert len(ml) == case["matches"]
    assert hashlib.md5(ml.text().encode()).hexdigest() == case["md5"]
    if "collisions" in case:
        assert st["collision_count"] == case["collisions"]


@pytest.mark.parametrize("G,n,w,p,table_size", [(3, 300_000, 13, 0.03, 40000), (4, 200_000, 15, 0.03, 7),
                                                (5, 200_000, 11, 0.02, 1), (6, 150_000, 15, 0.01, 40000)])
def test_big_bucket_replay_oracle(gpu_lib, oracle_mod, G, n, w, p, table_size, force_big):
    seqs = oracle_mod.generate(G, n, p, 77 + G + w)
    seed = oracle_mod.get_seed(w)
    lengths, starts, ref = oracle_mod.find_matches(seqs, seed, table_size=table_size)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        mh.SetTableSize(table_size)
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert st["collision_count"] == ref["collision_count"] and st["mem_count"] == ref["mem_count"]
