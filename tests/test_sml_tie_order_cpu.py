"""Order of equal seed mers in a SortedMerList (MemorySML::Create, MemorySML.cpp:45-60).

1. The oracle's SML (std_sort.h restatement of libstdc++ introsort) equals the real
   std::sort(bmer, &bmer_lessthan) of this toolchain on {position, mer} arrays filled in
   position order (tests/sml_sort_model.cpp), ties included.
2. On the inputs of tests/tie_inputs.py, FindMatches under the reference's tie order and
   under position order: the test reports how many inputs differ (every one of them runs
   on the GPU against the std::sort-order oracle in tests/test_gpu_tie_order.py).
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle
from tests import repeat_inputs, tie_inputs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "_build")
SO = os.path.join(BUILD, "libsml_sort_model.so")
REPORT = os.path.join(BUILD, "tie_order_report.json")


@pytest.fixture(scope="module")
def model():
    oracle.lib()
    os.makedirs(BUILD, exist_ok=True)
    odir = os.path.join(ROOT, "oracle", "build")
    tmp = f"{SO}.{os.getpid()}"   # build aside, then rename: parallel workers never load a partial file
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", tmp,
                    os.path.join(ROOT, "tests", "sml_sort_model.cpp"), f"-L{odir}", "-lmums_oracle",
                    f"-Wl,-rpath,{odir}"], check=True)
    os.replace(tmp, SO)
    L = ctypes.CDLL(SO)
    L.model_sml_positions.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    L.model_sml_positions.restype = ctypes.c_int64
    return L


def model_sml(L, seq, seed):
    out = np.zeros(max(len(seq), 1), dtype=np.uint32)
    m = L.model_sml_positions(seq, len(seq), seed, out.ctypes.data)
    assert m >= 0
    return out[:m]


def _pin(L, seqs, w):
    seed = oracle.get_seed(w)
    ties = 0
    for s in seqs:
        ref = model_sml(L, s, seed)
        got = oracle.build_sml(s, seed)
        assert np.array_equal(got, ref)
        keys = oracle.seed_keys(s, seed)[ref]
        ties += int(np.count_nonzero(keys[1:] == keys[:-1]))
    return ties


@pytest.mark.parametrize("name", sorted(tie_inputs.CASES))
def test_oracle_sml_equals_std_sort(model, name):
    gen, opts = tie_inputs.CASES[name]
    _pin(model, gen(), opts.get("w", 15))


@pytest.mark.parametrize("w", [9, 11, 15, 19, 21, 27, 31])
def test_oracle_sml_equals_std_sort_weights(model, w):
    seqs = repeat_inputs.n_gapped(G=2, n=40_000, gaps=((5_000, 2000), (20_000, 700)), seed=w)
    seqs += oracle.generate(1, 30_000, 0.0, w)
    assert _pin(model, seqs, w) > 0


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 30, 31, 33, 100])
def test_oracle_sml_equals_std_sort_short(model, n):
    # short sequences: the introsort loop does nothing below 17 records (final insertion sort only)
    rng = np.random.default_rng(n)
    for s in (b"A" * n, bytes(rng.choice(list(b"AC"), n)) if n else b"", bytes(rng.choice(list(b"ACGT"), n))):
        _pin(model, [s], 5)


def _matches(seqs, opts):
    ln, st, stats = oracle.find_matches(seqs, oracle.get_seed(opts.get("w", 15)), **tie_inputs.oracle_kwargs(opts))
    return oracle.match_text(ln, st), stats


def test_tie_rule_difference_report():
    """FindMatches under libstdc++'s tie order vs position order on every tie input."""
    differ, same = [], []
    for name in sorted(tie_inputs.CASES):
        gen, opts = tie_inputs.CASES[name]
        seqs = gen()
        with oracle.sml_tie_rule("std"):
            a, sa = _matches(seqs, opts)
        with oracle.sml_tie_rule("position"):
            b, sb = _matches(seqs, opts)
        if a != b or sa["offset_log"].tolist() != sb["offset_log"].tolist():
            differ.append(name)
        else:
            same.append(name)
    os.makedirs(BUILD, exist_ok=True)
    with open(REPORT, "w") as f:
        json.dump({"differ": differ, "same": same}, f, indent=1)
    print(f"\ntie order: {len(differ)} of {len(differ) + len(same)} inputs differ: {differ}")
    # the reference's order is observable through MER_REPEAT_LIMIT restarts (high-copy
    # repeats), ParallelMemHash chunk starts and the repeat tolerance's first copy
    assert {"high_copy_spread", "high_copy_tandem", "dup_block_compat_0", "tandem_rtol1_0",
            "dup_block_rtol1"} <= set(differ), differ
