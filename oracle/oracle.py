"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the C oracle (oracle/mums_oracle.c).

The oracle is the CPU restatement of libMems' MemHash path used to check the
HIP implementation.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module; the product (libmems_amd) never does.
Parity pinning: SURVEY.md Appendix C known-answer md5s (tests/test_oracle_pinning.py).
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import subprocess
from typing import Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libmums_oracle.so")
CLI = os.path.join(HERE, "build", "oracle_cli")

_lib = None


class _Params(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("repeat_tol", ctypes.c_uint32),
        ("enum_tol", ctypes.c_uint32),
        ("table_size", ctypes.c_uint32),
        ("masked", ctypes.c_int),
        ("seq_mask", ctypes.c_uint64),
        ("gnseqi_end_neg1", ctypes.c_int),
        ("seeds_only", ctypes.c_int),
        ("parallel_compat", ctypes.c_int),
        ("chunk_size", ctypes.c_uint64),
        ("pairwise", ctypes.c_int),
        ("start_points", ctypes.c_void_p),
    ]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, u64 = ctypes.c_void_p, ctypes.c_uint64
        L.oracle_get_seed.argtypes = [ctypes.c_int, ctypes.c_int]
        L.oracle_get_seed.restype = ctypes.c_int64
        L.oracle_seed_length.argtypes = [ctypes.c_int64]
        L.oracle_seed_weight.argtypes = [ctypes.c_int64]
        L.oracle_default_seed_weight.argtypes = [u64]
        L.oracle_default_seed_weight.restype = ctypes.c_uint
        L.oracle_pack.argtypes = [ctypes.c_char_p, u64, vp]
        L.oracle_pack.restype = ctypes.c_int64
        L.oracle_seed_keys.argtypes = [ctypes.c_char_p, u64, u64, vp]
        L.oracle_build_sml.argtypes = [ctypes.c_char_p, u64, u64, vp]
        L.oracle_find_matches.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(u64),
                                          ctypes.POINTER(_Params)]
        L.oracle_find_matches.restype = vp
        L.oracle_find_matches_omp.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(u64),
                                              ctypes.POINTER(_Params), ctypes.c_int]
        L.oracle_find_matches_omp.restype = vp
        L.oracle_omp_threads.restype = ctypes.c_int
        for f in ("count", "mem_count", "collision_count", "max_group", "probe_count", "seedmers", "chunks", "restarts"):
            fn = getattr(L, f"oracle_result_{f}")
            fn.argtypes = [vp]
            fn.restype = u64
        L.oracle_result_seqcount.argtypes = [vp]
        L.oracle_result_probe_log.argtypes = [vp, vp, vp]
        L.oracle_result_copy.argtypes = [vp, vp, vp]
        L.oracle_result_offset_log.argtypes = [vp, vp]
        L.oracle_result_free.argtypes = [vp]
        L.oracle_generate.argtypes = [ctypes.c_int, u64, ctypes.c_double, u64, ctypes.c_char_p]
        L.oracle_set_sml_tie_rule.argtypes = [ctypes.c_int]
        L.oracle_get_sml_tie_rule.restype = ctypes.c_int
        _lib = L
    return _lib


@contextlib.contextmanager
def sml_tie_rule(rule: str):
    """Order of equal seed mers in the oracle's SortedMerLists: "std" (libstdc++ std::sort,
    MemorySML.cpp:54 -- the reference and the default) or "position" (a stable sort's
    order, kept only to count the inputs on which the two rules differ)."""
    L = lib()
    old = L.oracle_get_sml_tie_rule()
    L.oracle_set_sml_tie_rule({"std": 1, "position": 0}[rule])
    try:
        yield
    finally:
        L.oracle_set_sml_tie_rule(old)


def get_seed(weight: int, rank: int = 0) -> int:
    return int(lib().oracle_get_seed(weight, rank)) & 0xFFFFFFFFFFFFFFFF


def generate(G: int, n: int, p: float, seed: int = 12345) -> list:
    """SURVEY.md Appendix C generator (std::mt19937_64)."""
    buf = ctypes.create_string_buffer(G * n)
    lib().oracle_generate(G, n, p, seed, buf)
    raw = buf.raw
    return [raw[g * n:(g + 1) * n] for g in range(G)]


def pack(seq: bytes) -> np.ndarray:
    nw = (2 * len(seq)) // 32 + (1 if (2 * len(seq)) % 32 else 0) + 2
    out = np.zeros(nw, dtype=np.uint32)
    rc = lib().oracle_pack(seq, len(seq), out.ctypes.data)
    if rc < 0:
        raise ValueError("gap in sequence")
    return out


def seed_keys(seq: bytes, seed: int) -> np.ndarray:
    L = lib().oracle_seed_length(seed)
    m = max(len(seq) - L + 1, 0)
    out = np.zeros(max(m, 1), dtype=np.uint64)
    lib().oracle_seed_keys(seq, len(seq), seed, out.ctypes.data)
    return out[:m]


def build_sml(seq: bytes, seed: int) -> np.ndarray:
    L = lib().oracle_seed_length(seed)
    m = max(len(seq) - L + 1, 0)
    out = np.zeros(max(m, 1), dtype=np.uint32)
    lib().oracle_build_sml(seq, len(seq), seed, out.ctypes.data)
    return out[:m]


def seed_occurrence(seq: bytes, seed: int) -> np.ndarray:
    """SeedOccurrenceList::construct (SeedOccurrenceList.h:22-87): float32 per position."""
    out = np.zeros(max(len(seq), 1), dtype=np.float32)
    lib().oracle_seed_occurrence.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    rc = lib().oracle_seed_occurrence(seq, len(seq), seed, out.ctypes.data)
    if rc:
        raise ValueError("oracle rejected input")
    return out[:len(seq)]


def find_matches(seqs: Sequence[bytes], seed: int, repeat_tol: int = 0, enum_tol: int = 1,
                 table_size: int = 40000, masked: bool = False, seq_mask: int = 0,
                 gnseqi_end_neg1: bool = False, seeds_only: bool = False, parallel_compat: bool = False,
                 chunk_size: int = 0, pairwise: bool = False,
                 start_points: Sequence[int] | None = None,
                 omp_threads: int | None = None) -> Tuple[np.ndarray, np.ndarray, dict]:
    """MemHash::FindMatches restated; returns (lengths[M], starts[M,G], counters).
    parallel_compat: ParallelMemHash::FindMatches instead (ParallelMemHash.cpp:42-121),
    chunk_size = its CHUNK_SIZE (0 = 200000).  start_points: FindMatchesFromPosition
    (MemHash.cpp:117-127) start SML index per genome.  omp_threads: run the OpenMP driver
    (oracle_find_matches_omp, same result) on that many threads (0 = OpenMP default)."""
    G = len(seqs)
    arr = (ctypes.c_char_p * G)(*seqs)
    lens = (ctypes.c_uint64 * G)(*[len(s) for s in seqs])
    sp = None
    if start_points is not None:
        sp = (ctypes.c_uint64 * G)(*[int(x) for x in start_points])
    prm = _Params(seed, repeat_tol, enum_tol, table_size, int(masked), seq_mask, int(gnseqi_end_neg1),
                  int(seeds_only), int(parallel_compat), chunk_size, int(pairwise),
                  ctypes.cast(sp, ctypes.c_void_p) if sp is not None else None)
    L = lib()
    if omp_threads is None:
        r = L.oracle_find_matches(G, arr, lens, ctypes.byref(prm))
    else:
        r = L.oracle_find_matches_omp(G, arr, lens, ctypes.byref(prm), int(omp_threads))
    if not r:
        raise ValueError("oracle rejected input")
    try:
        c = L.oracle_result_count(r)
        lengths = np.zeros(c, dtype=np.uint64)
        starts = np.zeros((c, G), dtype=np.int64)
        if c:
            L.oracle_result_copy(r, lengths.ctypes.data, starts.ctypes.data)
        stats = dict(mem_count=L.oracle_result_mem_count(r), collision_count=L.oracle_result_collision_count(r),
                     max_group=L.oracle_result_max_group(r), probes=L.oracle_result_probe_count(r),
                     seedmers=L.oracle_result_seedmers(r), chunks=L.oracle_result_chunks(r),
                     restarts=L.oracle_result_restarts(r))
        offlog = np.zeros((int(stats["restarts"]), G), dtype=np.uint64)
        if stats["restarts"] and not parallel_compat:
            L.oracle_result_offset_log(r, offlog.ctypes.data)
        stats["offset_log"] = offlog
        L.oracle_result_progress.restype = ctypes.c_char_p
        L.oracle_result_progress.argtypes = [ctypes.c_void_p]
        stats["progress"] = (L.oracle_result_progress(r) or b"").decode()
        L.oracle_result_match_log.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_result_match_log_count.restype = ctypes.c_uint64
        L.oracle_result_match_log_count.argtypes = [ctypes.c_void_p]
        nlog = int(L.oracle_result_match_log_count(r))
        ml_len = np.zeros(nlog, dtype=np.uint64)
        ml_s = np.zeros((nlog, G), dtype=np.int64)
        if L.oracle_result_match_log(r, ml_len.ctypes.data, ml_s.ctypes.data) == 0:
            stats["match_log"] = (ml_len, ml_s)   # SetMatchLog: inserted entries in insertion order
    finally:
        L.oracle_result_free(r)
    return lengths, starts, stats


def replay_rows(seqs: Sequence[bytes], seed: int, rows: np.ndarray, table_size: int = 40000):
    """AddHashEntry replay (extension + bucket insertion) of given probe rows
    {starts[G], offset} in order; returns (lengths, starts, counters) like find_matches."""
    G = len(seqs)
    arr = (ctypes.c_char_p * G)(*seqs)
    lens = (ctypes.c_uint64 * G)(*[len(s) for s in seqs])
    prm = _Params(seed, 0, 1, table_size, 0, 0, 0, 0)
    rows = np.ascontiguousarray(rows, dtype=np.int64).reshape(-1, G + 1)
    L = lib()
    L.oracle_replay_rows.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.POINTER(_Params), ctypes.c_void_p, ctypes.c_uint64]
    L.oracle_replay_rows.restype = ctypes.c_void_p
    r = L.oracle_replay_rows(G, arr, lens, ctypes.byref(prm), rows.ctypes.data, rows.shape[0])
    if not r:
        raise ValueError("oracle rejected input")
    try:
        c = L.oracle_result_count(r)
        lengths = np.zeros(c, dtype=np.uint64)
        starts = np.zeros((c, G), dtype=np.int64)
        if c:
            L.oracle_result_copy(r, lengths.ctypes.data, starts.ctypes.data)
        stats = dict(mem_count=L.oracle_result_mem_count(r), collision_count=L.oracle_result_collision_count(r))
    finally:
        L.oracle_result_free(r)
    return lengths, starts, stats


def seed_probes(seqs: Sequence[bytes], seed: int, table_size: int = 40000, parallel_compat: bool = False,
                chunk_size: int = 0, omp_threads: int | None = None) -> Tuple[np.ndarray, np.ndarray, dict]:
    """Seed stage only (keys, SMLs, G-way merge, acceptance, probes): the AddHashEntry calls
    in order as (bucket[P], ref[P]) with ref = global seed-mer index of the probe's first
    start (genome bases = cumulative SMLLength), plus the counters."""
    G = len(seqs)
    arr = (ctypes.c_char_p * G)(*seqs)
    lens = (ctypes.c_uint64 * G)(*[len(s) for s in seqs])
    prm = _Params(seed, 0, 1, table_size, 0, 0, 0, 1, int(parallel_compat), chunk_size)
    L = lib()
    if omp_threads is None:
        r = L.oracle_find_matches(G, arr, lens, ctypes.byref(prm))
    else:
        r = L.oracle_find_matches_omp(G, arr, lens, ctypes.byref(prm), int(omp_threads))
    if not r:
        raise ValueError("oracle rejected input")
    try:
        P = L.oracle_result_probe_count(r)
        b = np.zeros(max(P, 1), dtype=np.uint32)
        ref = np.zeros(max(P, 1), dtype=np.uint64)
        if P:
            L.oracle_result_probe_log(r, b.ctypes.data, ref.ctypes.data)
        stats = dict(probes=P, seedmers=L.oracle_result_seedmers(r), max_group=L.oracle_result_max_group(r))
    finally:
        L.oracle_result_free(r)
    return b[:P], ref[:P], stats


def match_text(lengths: np.ndarray, starts: np.ndarray) -> str:
    if len(lengths) == 0:
        return ""
    arr = np.concatenate([lengths.astype(np.int64)[:, None], starts], axis=1)
    return "".join("\t".join(map(str, row)) + "\n" for row in arr.tolist())


def eliminate_overlaps(lengths: np.ndarray, starts: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """EliminateOverlaps (Aligner.cpp:62-176) of a MatchList (lengths [M], starts [M, G])."""
    L = lib()
    u64 = ctypes.c_uint64
    L.oracle_eliminate_overlaps.argtypes = [ctypes.c_int, u64, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.POINTER(ctypes.POINTER(u64)),
                                            ctypes.POINTER(ctypes.POINTER(ctypes.c_int64))]
    L.oracle_eliminate_overlaps.restype = u64
    L.oracle_free.argtypes = [ctypes.c_void_p]
    lengths = np.ascontiguousarray(lengths, dtype=np.uint64)
    starts = np.ascontiguousarray(starts, dtype=np.int64)
    M, G = starts.shape
    lo = ctypes.POINTER(u64)()
    so = ctypes.POINTER(ctypes.c_int64)()
    n = L.oracle_eliminate_overlaps(G, M, lengths.ctypes.data, starts.ctypes.data, ctypes.byref(lo), ctypes.byref(so))
    out_l = np.ctypeslib.as_array(lo, shape=(max(n, 1),))[:n].copy()
    out_s = np.ctypeslib.as_array(so, shape=(max(n, 1) * G,))[:n * G].reshape(n, G).copy()
    L.oracle_free(ctypes.cast(lo, ctypes.c_void_p))
    L.oracle_free(ctypes.cast(so, ctypes.c_void_p))
    return out_l, out_s


def std_sort_ids(keys: np.ndarray, depth: int = -1) -> np.ndarray:
    """libstdc++ std::sort of ids 0..n-1 by keys[id] (restated), optional depth override."""
    L = lib()
    L.oracle_std_sort_ids.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    L.oracle_std_sort_depth_override.argtypes = [ctypes.c_int]
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    ids = np.arange(len(keys), dtype=np.uint32)
    L.oracle_std_sort_depth_override(depth)
    try:
        L.oracle_std_sort_ids(ids.ctypes.data, len(keys), keys.ctypes.data)
    finally:
        L.oracle_std_sort_depth_override(-1)
    return ids


def compat_rank_table(seqs: Sequence[bytes], seed: int, chunk_size: int, rank: int, ranks: int,
                      table_size: int = 40000) -> Tuple[np.ndarray, np.ndarray, dict]:
    """One rank of the chunk-range model: ParallelMemHash::FindMatches on the
    chunks [nch * rank / ranks, nch * (rank + 1) / ranks) from empty tables; its table in
    bucket order (oracle parallel_compat = 4096 + (ranks << 8) + rank)."""
    assert 1 <= ranks < 256 and 0 <= rank < ranks
    return find_matches(seqs, seed, table_size=table_size, parallel_compat=4096 + (ranks << 8) + rank,
                        chunk_size=chunk_size)


def merge_tables(tables: Sequence[Tuple[np.ndarray, np.ndarray]], G: int,
                 table_size: int = 40000) -> Tuple[np.ndarray, np.ndarray, dict]:
    """MergeTable (ParallelMemHash.cpp:105-121) of the given tables (lengths, starts; each in
    bucket / vector order) into one empty table, table after table (oracle_merge_tables)."""
    L = lib()
    L.oracle_merge_tables.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint32]
    L.oracle_merge_tables.restype = ctypes.c_void_p
    lens = np.ascontiguousarray(np.concatenate([np.asarray(t[0], dtype=np.uint64) for t in tables] or
                                               [np.zeros(0, np.uint64)]))
    sts = np.ascontiguousarray(np.concatenate([np.asarray(t[1], dtype=np.int64).reshape(-1, G) for t in tables] or
                                              [np.zeros((0, G), np.int64)]))
    nrows = np.array([len(t[0]) for t in tables] or [0], dtype=np.uint64)
    r = L.oracle_merge_tables(G, table_size, lens.ctypes.data, sts.ctypes.data, nrows.ctypes.data, len(tables))
    if not r:
        raise ValueError("oracle rejected input")
    try:
        c = L.oracle_result_count(r)
        lengths = np.zeros(c, dtype=np.uint64)
        starts = np.zeros((c, G), dtype=np.int64)
        if c:
            L.oracle_result_copy(r, lengths.ctypes.data, starts.ctypes.data)
        stats = dict(mem_count=L.oracle_result_mem_count(r), collision_count=L.oracle_result_collision_count(r))
    finally:
        L.oracle_result_free(r)
    return lengths, starts, stats


def entry_buckets(lengths: np.ndarray, starts: np.ndarray, table_size: int = 40000) -> np.ndarray:
    """Hash bucket of stored entries: CalculateOffset (MatchHashEntry.cpp:141-160) relative to
    the first start, mod table_size (MemHash.cpp:213)."""
    s = np.asarray(starts, dtype=np.int64)
    if s.size == 0:
        return np.zeros(0, dtype=np.int64)
    ln = np.asarray(lengths, dtype=np.int64)
    first = np.argmax(s != 0, axis=1)
    ref = s[np.arange(len(s)), first]
    cols = np.arange(s.shape[1])[None, :]
    t = s - ref[:, None] - np.where(s < 0, ln[:, None], 0)
    off = np.where((s != 0) & (cols > first[:, None]), t, 0).sum(axis=1)
    return ((off % table_size) + table_size) % table_size
