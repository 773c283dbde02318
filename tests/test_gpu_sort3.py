"""The three-pass seed sort (radix_wide.hip, MUMS_DEV_SORT3 = block shape 1/2/3): the 8-bit
MSD scatter, three 10-bit onesweep passes over key bits 1-30 and the parity bit unsorted under
the default tolerances (seg_parity_fix restores the SML order before a MER_REPEAT_LIMIT
restart; other tolerances keep the four 8-bit passes).  Every MatchList must equal the
reference's known answers / the oracle's, bit for bit."""
import hashlib
import json
import os

import pytest

from conftest import GOLDEN
from tests import repeat_inputs, tie_inputs

pytestmark = pytest.mark.gpu

CASES = [c for c in json.load(open(os.path.join(GOLDEN, "appendix_c.json")))["cases"]
         if c["mode"] != "ParallelMemHash" and not c.get("large")]


@pytest.mark.parametrize("shape", ["1", "2", "3"])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}_{c['mode']}")
def test_sort3_known_answers(gpu_lib, oracle_mod, monkeypatch, case, shape):
    monkeypatch.setenv("MUMS_DEV_SORT3", shape)
    seqs = oracle_mod.generate(case["G"], case["n"], case["p"], 12345)
    masked = case["mode"] == "MaskedMemHash"
    cls = gpu_lib.MaskedMemHash if masked else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(case["w"]))
        if masked:
            mh.SetMask(case.get("mask", 0))
        ml = mh.FindMatches(seqs)
        st = mh.stats()
    assert len(ml) == case["matches"]
    assert hashlib.md5(ml.text().encode()).hexdigest() == case["md5"]
    if "collisions" in case:
        assert st["collision_count"] == case["collisions"]
    if 2 * case["w"] + 1 <= 39:
        assert st["sort_passes"] == 3


def _vs_oracle(gpu_lib, oracle_mod, seqs, w, start_points=None, repeat_tol=0):
    seed = oracle_mod.get_seed(w)
    with oracle_mod.sml_tie_rule("std"):
        lengths, starts, ost = oracle_mod.find_matches(seqs, seed, start_points=start_points, repeat_tol=repeat_tol)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        mh.SetRepeatTolerance(repeat_tol)
        ml = mh.FindMatchesFromPosition(seqs, start_points) if start_points is not None else mh.FindMatches(seqs)
        st = mh.stats()
    assert st["restarts"] == ost["restarts"]
    assert len(ml) == len(lengths)
    assert (ml.lengths == lengths).all() and (ml.starts == starts).all()
    assert st["collision_count"] == ost["collision_count"]
    return st, ost


@pytest.mark.parametrize("w", [15, 17, 19])
def test_sort3_restarts(gpu_lib, oracle_mod, monkeypatch, w):
    """N runs: MER_REPEAT_LIMIT restarts on a parity-masked stream (seg_parity_fix first)."""
    monkeypatch.setenv("MUMS_DEV_SORT3", "1")
    seqs = repeat_inputs.n_gapped(G=3, n=200_000, gaps=((40_000, 3000), (120_000, 3000)), shift=500, seed=1)
    st, ost = _vs_oracle(gpu_lib, oracle_mod, seqs, w)
    assert ost["restarts"] > 0


DEFAULT_TOL = sorted(k for k, (gen, o) in tie_inputs.CASES.items()
                     if o.get("repeat_tol", 0) == 0 and o.get("enum_tol", 1) == 1 and o.get("w", 15) <= 19
                     and not o.get("cls"))


@pytest.mark.parametrize("name", DEFAULT_TOL)
def test_sort3_tie_inputs(gpu_lib, oracle_mod, monkeypatch, name):
    """Gap-boundary ties, start points inside runs of equal keys, high-copy restarts."""
    from tests.test_gpu_tie_order import run_case
    monkeypatch.setenv("MUMS_DEV_SORT3", "2")
    gen, opts = tie_inputs.CASES[name]
    seqs = gen()
    with oracle_mod.sml_tie_rule("std"):
        ref_len, ref_starts, ref = oracle_mod.find_matches(seqs, oracle_mod.get_seed(opts.get("w", 15)),
                                                           **tie_inputs.oracle_kwargs(opts))
    ml, st, offlog = run_case(gpu_lib, seqs, opts)
    assert len(ml) == len(ref_len), (len(ml), len(ref_len))
    assert (ml.lengths == ref_len).all() and (ml.starts == ref_starts).all()


@pytest.mark.parametrize("w", [15, 19])
def test_sort3_sorted_mer_lists(gpu_lib, oracle_mod, monkeypatch, w):
    """mums_build_sml (the deferred SML's materialisation) after a three-pass seed stage:
    every genome's SML in std::sort order."""
    import numpy as np
    monkeypatch.setenv("MUMS_DEV_SORT3", "1")
    seqs = tie_inputs.multi_gap(seed=3)
    seed = oracle_mod.get_seed(w)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        for sq in seqs:
            mh.AddSequence(sq)
        mh.FindStage(gpu_lib.STAGE_SEEDS)
        for g, sq in enumerate(seqs):
            with oracle_mod.sml_tie_rule("std"):
                ref = oracle_mod.build_sml(sq, seed)
            assert np.array_equal(mh.SortedMerList(g, len(ref)), ref)


def test_sort3_start_points_and_repeat_tol(gpu_lib, oracle_mod, monkeypatch):
    """Start points (parity fix before the plan) and repeat tolerance (four 8-bit passes)."""
    monkeypatch.setenv("MUMS_DEV_SORT3", "3")
    seqs = repeat_inputs.n_gapped(G=4, n=90_000, gaps=((2_000, 25_000), (60_000, 4_000)), shift=1_300, seed=31)
    _vs_oracle(gpu_lib, oracle_mod, seqs, 15, start_points=[3, 9_999, 10_001, 40_000])
    seqs = oracle_mod.generate(3, 200_000, 0.02, 5)
    _vs_oracle(gpu_lib, oracle_mod, seqs, 15, repeat_tol=2)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"G{c['G']}_n{c['n']}_p{c['p']}_{c['mode']}")
def test_xcd_claim_queues_known_answers(gpu_lib, oracle_mod, monkeypatch, case):
    """The four-pass sort with XCD-grouped claim queues (MUMS_DEV_OS_XCD: bucket b's tiles in
    queue b % 8, blocks claim from queue blockIdx % 8 first, then steal): same MatchList."""
    monkeypatch.setenv("MUMS_DEV_OS_XCD", "1")
    seqs = oracle_mod.generate(case["G"], case["n"], case["p"], 12345)
    masked = case["mode"] == "MaskedMemHash"
    cls = gpu_lib.MaskedMemHash if masked else gpu_lib.MemHash
    with cls(0) as mh:
        mh.SetSeed(oracle_mod.get_seed(case["w"]))
        if masked:
            mh.SetMask(case.get("mask", 0))
        ml = mh.FindMatches(seqs)
    assert len(ml) == case["matches"]
    assert hashlib.md5(ml.text().encode()).hexdigest() == case["md5"]
