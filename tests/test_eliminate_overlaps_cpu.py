"""EliminateOverlaps (Aligner.cpp:62-176), CPU side: the oracle's restatement of libstdc++'s
std::sort (introsort: tie order of SingleStartComparator) against the real std::sort /
std::partial_sort of this toolchain, and the oracle's EliminateOverlaps against a C++ model
over Match* vectors sorted by the real std::sort (tests/eo_model.cpp)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "_build")
SO = os.path.join(BUILD, "libeo_model.so")


@pytest.fixture(scope="module")
def model():
    os.makedirs(BUILD, exist_ok=True)
    tmp = f"{SO}.{os.getpid()}"   # build aside, then rename: parallel workers never load a partial file
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", tmp, os.path.join(ROOT, "tests", "eo_model.cpp")],
                   check=True)
    os.replace(tmp, SO)
    L = ctypes.CDLL(SO)
    L.model_std_sort.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    L.model_eliminate_overlaps.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    L.model_eliminate_overlaps.restype = ctypes.c_uint64
    return L


def model_sort(L, keys, heap_only=False):
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    ids = np.arange(len(keys), dtype=np.uint32)
    L.model_std_sort(ids.ctypes.data, len(keys), keys.ctypes.data, int(heap_only))
    return ids


@pytest.mark.parametrize("n", [0, 1, 2, 15, 16, 17, 18, 33, 100, 1000, 5000, 40000])
@pytest.mark.parametrize("span", [1, 3, 50, 1 << 40])
def test_std_sort_restatement_matches_libstdcxx(model, n, span):
    rng = np.random.default_rng(n * 7 + span % 1000)
    keys = rng.integers(0, span, size=n, dtype=np.uint64)
    if n > 10:
        keys[rng.integers(0, n, size=n // 3)] = 0      # NO_MATCH group
    assert np.array_equal(oracle.std_sort_ids(keys), model_sort(model, keys))


@pytest.mark.parametrize("n", [17, 64, 1000, 4097])
def test_heap_fallback_matches_partial_sort(model, n):
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 20, size=n, dtype=np.uint64)
    assert np.array_equal(oracle.std_sort_ids(keys, depth=0), model_sort(model, keys, heap_only=True))


def random_matchlist(rng, M, G, n=20000, max_len=300, p_absent=0.3, p_rev=0.3, start_span=None):
    """Matches with overlaps, reverse components, NO_MATCH and tied starts."""
    span = start_span or n
    lengths = rng.integers(1, max_len, size=M).astype(np.uint64)
    starts = rng.integers(1, span, size=(M, G)).astype(np.int64)
    starts[rng.random((M, G)) < p_rev] *= -1
    starts[rng.random((M, G)) < p_absent] = 0
    starts[:, 0] = np.where(starts[:, 0] == 0, 1 + rng.integers(0, span, size=M), starts[:, 0])
    return lengths, starts


def model_eo(L, lengths, starts):
    M, G = starts.shape
    cap = 8 * M + 64
    lo = np.zeros(cap, dtype=np.uint64)
    so = np.zeros(cap * G, dtype=np.int64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    k = L.model_eliminate_overlaps(G, M, lengths.ctypes.data, starts.ctypes.data, lo.ctypes.data, so.ctypes.data, cap)
    assert k <= cap
    return lo[:k], so[:k * G].reshape(k, G)


@pytest.mark.parametrize("M,G,span,seed", [(2, 2, 50, 1), (10, 2, 100, 2), (200, 3, 2000, 3), (3000, 4, 30000, 4),
                                           (5000, 8, 20000, 5), (20000, 5, 400000, 6), (3000, 3, 300, 7)])
def test_eliminate_overlaps_oracle_matches_model(model, M, G, span, seed):
    rng = np.random.default_rng(seed)
    lengths, starts = random_matchlist(rng, M, G, start_span=span)
    ol, os_ = oracle.eliminate_overlaps(lengths, starts)
    ml, ms = model_eo(model, lengths, starts)
    assert np.array_equal(ol, ml) and np.array_equal(os_, ms)


def test_eliminate_overlaps_on_findmatches_output(model):
    # repeat-rich related genomes: MemHash MatchLists with overlapping entries
    seqs = oracle.generate(4, 400_000, 0.02, 99)
    rep = seqs[0][1000:3000]
    seqs = [s[:50_000] + rep + s[50_000:200_000] + rep + s[200_000:] for s in seqs]
    lengths, starts, _ = oracle.find_matches(seqs, oracle.get_seed(11))
    ol, os_ = oracle.eliminate_overlaps(lengths, starts)
    ml, ms = model_eo(model, lengths, starts)
    assert len(ol) != len(lengths) or not np.array_equal(os_, starts)   # something was cropped
    assert np.array_equal(ol, ml) and np.array_equal(os_, ms)
