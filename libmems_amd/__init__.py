"""libmems_amd -- MI355X-native multi-MUM seed finder (libMems MemHash hot path).

Python mirror of the reference's MemHash / MaskedMemHash interface
(koadman/libMems 1.6.1, libMems/MemHash.h:38-175, MaskedMemHash.h:25-40) over
the C ABI in include/mums.h (libmums_hip.so, built in-tree by `make -C
libmems_amd`).  All compute runs in hand-written HIP kernels for gfx950; there
is no CPU fallback: if the shared library or a HIP device is missing, the
calls raise instead of computing anything on the host.

Method names follow the reference (AddSequence, FindMatches, GetMatchList,
SetRepeatTolerance, SetEnumerationTolerance, SetTableSize, MemCount,
MemCollisionCount, Clear, SetMask) so parity tests read like the reference's
usage in Aligner.cpp:1181-1207.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MUMS_DEV_LIB: development builds of the same sources (libmems_amd/Makefile EXTRA=...)
LIB_PATH = os.environ.get("MUMS_DEV_LIB") or os.path.join(_HERE, "libmums_hip.so")

MUMS_OK = 0
MUMS_E_INVALID = -1
MUMS_E_NOMEM = -2
MUMS_E_HIP = -3
MUMS_E_GAP = -4
MUMS_E_UNSUPPORTED = -5
MUMS_E_NODEVICE = -6

STAGE_SEEDS = 1
STAGE_ALL = 2

DEFAULT_MEM_TABLE_SIZE = 40000       # MemHash.h:30
DEFAULT_REPEAT_TOLERANCE = 0         # MemHash.h:31
DEFAULT_ENUMERATION_TOLERANCE = 1    # MemHash.h:32
SOLID_SEED = 2147483647              # SeedMasks.h:263


class MumsError(RuntimeError):
    """A non-zero status from the C ABI (the reference would have thrown)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"mums error {code}: {msg}")
        self.code = code


class GapInSequence(MumsError):
    """SortedMerList.cpp:433-437 throws "Gap in genome sequence"."""


class _Stats(ctypes.Structure):
    _fields_ = [
        ("seedmers", ctypes.c_uint64),
        ("groups", ctypes.c_uint64),
        ("probes", ctypes.c_uint64),
        ("mem_count", ctypes.c_uint64),
        ("collision_count", ctypes.c_uint64),
        ("repeat_limit_groups", ctypes.c_uint64),
        ("nonempty_buckets", ctypes.c_uint64),
        ("ms_keys", ctypes.c_double),
        ("ms_sort", ctypes.c_double),
        ("ms_groups", ctypes.c_double),
        ("ms_buckets", ctypes.c_double),
        ("ms_replay", ctypes.c_double),
        ("ms_output", ctypes.c_double),
        ("ms_total", ctypes.c_double),
        ("ms_dominant", ctypes.c_double),
        ("dominant_launches", ctypes.c_uint64),
        ("dominant_bytes", ctypes.c_uint64),
        ("key_bytes", ctypes.c_uint64),
        ("sort_passes", ctypes.c_uint64),
        ("ms_chains", ctypes.c_double),
        ("chains", ctypes.c_uint64),
        ("chunks", ctypes.c_uint64),
        ("restarts", ctypes.c_uint64),
        ("ms_chain_walks", ctypes.c_double),
        ("chain_walk_words", ctypes.c_uint64),
        ("chain_walks", ctypes.c_uint64),
        ("chain_walk_bytes", ctypes.c_uint64),
        ("ms_short_walks", ctypes.c_double),
        ("short_walk_words", ctypes.c_uint64),
        ("short_walks", ctypes.c_uint64),
        ("short_walk_bytes", ctypes.c_uint64),
    ]


EXPORTED_SYMBOLS = [
    "mums_abi_version", "mums_ctx_create", "mums_ctx_destroy", "mums_set_stream", "mums_set_seed",
    "mums_set_params", "mums_set_mask", "mums_add_genome", "mums_add_genome_device", "mums_clear",
    "mums_find", "mums_find_stage", "mums_result_count", "mums_result_copy", "mums_get_stats",
    "mums_last_error", "mums_get_seed", "mums_default_seed_weight", "mums_copy_seed_keys",
    "mums_build_sml", "mums_set_profiling", "mums_shard_layout", "mums_shard_msd_bits", "mums_shard_keys",
    "mums_shard_merge", "mums_probe_count", "mums_probe_copy", "mums_shard_bucket_counts", "mums_shard_probe_rows",
    "mums_shard_packed_info", "mums_shard_packed_copy", "mums_shard_find", "mums_set_parallel_compat",
    "mums_seed_occurrence", "mums_multiplicity_filter", "mums_length_filter", "mums_write_sml",
    "mums_add_genome_sml", "mums_set_pairwise", "mums_shard_slice", "mums_set_start_points",
    "mums_get_offset_log", "mums_copy_seed_keys_range", "mums_mem_table_count", "mums_eliminate_overlaps",
    "mums_load_matches", "mums_debug_std_sort", "mums_comm_unique_id", "mums_comm_init_rank", "mums_comm_init_all",
    "mums_comm_init_local", "mums_comm_destroy", "mums_comm_last_error", "mums_shard_key_ranges", "mums_shard_run",
    "mums_set_match_log", "mums_match_log_copy", "mums_shard_restart_pending", "mums_shard_stream",
    "mums_shard_restart_plan", "mums_shard_restart_apply", "mums_comm_init_host", "mums_set_progress_log",
    "mums_progress_log_copy", "mums_shard_restart_counts", "mums_shard_restart_prepare", "mums_shard_restart_step",
    "mums_shard_restart_log", "mums_shard_restart_runs", "mums_shard_restart_ties", "mums_shard_restart_finish",
    "mums_shard_restart_info", "mums_shard_tie_flags", "mums_shard_tie_replay", "mums_shard_tie_apply",
    "mums_genome_device", "mums_shard_chain_label", "mums_shard_chain_export", "mums_shard_find_labelled",
    "mums_shard_chain_info", "mums_shard_chain_entries", "mums_shard_entry_thresholds", "mums_shard_kept_export",
    "mums_shard_find_kept", "mums_comm_exchange_info",
]

# mums_comm_ops (include/mums.h): the caller's transport as two host callbacks
COMM_ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64,
                                     ctypes.POINTER(ctypes.c_uint64))
COMM_ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                     ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))


class MumsCommOps(ctypes.Structure):
    _fields_ = [("allgather_u64", COMM_ALLGATHER_FN), ("alltoallv", COMM_ALLTOALLV_FN)]

_lib: Optional[ctypes.CDLL] = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libmums_hip.so (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} not built: run `make -C {_HERE}` (hipcc --offload-arch=gfx950)")
    # PyTorch-ROCm ships its own libamdhip64.so.7 (same soname as /opt/rocm's).  Load it
    # first so this library binds to that one runtime instead of a second HIP/HSA runtime
    # in the same process (two runtimes cannot share the device).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.mums_abi_version.restype = i32
    lib.mums_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    lib.mums_ctx_destroy.argtypes = [vp]
    lib.mums_set_stream.argtypes = [vp, vp]
    lib.mums_set_seed.argtypes = [vp, u64]
    lib.mums_set_params.argtypes = [vp, u32, u32, u32]
    lib.mums_set_mask.argtypes = [vp, i32, u64]
    lib.mums_add_genome.argtypes = [vp, ctypes.c_char_p, u64]
    lib.mums_add_genome_device.argtypes = [vp, vp, u64]
    lib.mums_genome_device.argtypes = [vp, u32, ctypes.POINTER(vp), ctypes.POINTER(u64)]
    lib.mums_shard_chain_label.argtypes = [vp, vp, vp]
    lib.mums_shard_chain_export.argtypes = [vp, u32, vp, vp, vp, u64, vp, vp, u64, vp, vp]
    lib.mums_shard_find_labelled.argtypes = [vp, vp, vp, u64, vp, vp, u64, u32, vp, vp, vp]
    lib.mums_shard_chain_info.argtypes = [vp, vp]
    lib.mums_shard_chain_entries.argtypes = [vp, u32, vp, vp, u64, vp]
    lib.mums_shard_entry_thresholds.argtypes = [vp, vp, u64, vp]
    lib.mums_shard_kept_export.argtypes = [vp, u32, vp, vp, vp, u64, vp, vp, vp]
    lib.mums_shard_find_kept.argtypes = [vp, vp, vp, u64, vp, vp, u64, u32, vp, vp, u64, vp]
    lib.mums_comm_exchange_info.argtypes = [vp, vp]
    lib.mums_clear.argtypes = [vp]
    lib.mums_find.argtypes = [vp]
    lib.mums_find_stage.argtypes = [vp, i32]
    lib.mums_result_count.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u32)]
    lib.mums_result_copy.argtypes = [vp, vp, vp]
    lib.mums_get_stats.argtypes = [vp, ctypes.POINTER(_Stats)]
    lib.mums_last_error.argtypes = [vp]
    lib.mums_last_error.restype = ctypes.c_char_p
    lib.mums_get_seed.argtypes = [i32, i32]
    lib.mums_get_seed.restype = ctypes.c_int64
    lib.mums_default_seed_weight.argtypes = [u64]
    lib.mums_default_seed_weight.restype = u32
    lib.mums_copy_seed_keys.argtypes = [vp, u32, vp, u64]
    lib.mums_build_sml.argtypes = [vp, u32, vp, u64]
    lib.mums_set_profiling.argtypes = [vp, i32]
    lib.mums_shard_layout.argtypes = [vp, u32, u32, vp]
    lib.mums_shard_msd_bits.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u64)]
    lib.mums_shard_keys.argtypes = [vp, vp, u64, vp]
    lib.mums_shard_merge.argtypes = [vp, vp, u32, u32, u32, vp]
    lib.mums_probe_count.argtypes = [vp, ctypes.POINTER(u64)]
    lib.mums_probe_copy.argtypes = [vp, vp, vp, u64]
    lib.mums_shard_bucket_counts.argtypes = [vp, vp]
    lib.mums_shard_probe_rows.argtypes = [vp, u32, vp, vp, u64, vp]
    lib.mums_shard_packed_info.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.mums_shard_packed_copy.argtypes = [vp, vp]
    lib.mums_shard_find.argtypes = [vp, vp, u64, vp]
    lib.mums_set_parallel_compat.argtypes = [vp, i32, u64]
    lib.mums_seed_occurrence.argtypes = [vp, u32, vp, u64]
    lib.mums_multiplicity_filter.argtypes = [vp, u32]
    lib.mums_length_filter.argtypes = [vp, u64]
    lib.mums_write_sml.argtypes = [vp, u32, ctypes.c_char_p, ctypes.c_char_p]
    lib.mums_add_genome_sml.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(u64)]
    lib.mums_set_pairwise.argtypes = [vp, i32]
    lib.mums_shard_slice.argtypes = [vp, u32, vp, u32, u64, u64]
    lib.mums_set_start_points.argtypes = [vp, vp, u32]
    lib.mums_copy_seed_keys_range.argtypes = [vp, u32, u64, u64, vp]
    lib.mums_mem_table_count.argtypes = [vp, vp, u32]
    lib.mums_get_offset_log.argtypes = [vp, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(u32)]
    lib.mums_eliminate_overlaps.argtypes = [vp]
    lib.mums_load_matches.argtypes = [vp, u32, u64, vp, vp]
    lib.mums_debug_std_sort.argtypes = [vp, vp, u64, ctypes.c_int, vp]
    lib.mums_comm_unique_id.argtypes = [vp, u64]
    lib.mums_comm_init_rank.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, ctypes.c_int, vp]
    lib.mums_comm_init_all.argtypes = [ctypes.POINTER(vp), ctypes.c_int, vp]
    lib.mums_comm_init_local.argtypes = [ctypes.POINTER(vp), ctypes.c_int, vp]
    lib.mums_comm_init_host.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(MumsCommOps), vp]
    lib.mums_comm_destroy.argtypes = [vp]
    lib.mums_comm_destroy.restype = None
    lib.mums_comm_last_error.argtypes = [vp]
    lib.mums_comm_last_error.restype = ctypes.c_char_p
    lib.mums_shard_key_ranges.argtypes = [vp, u32, u32, vp, vp]
    lib.mums_shard_run.argtypes = [vp, vp, ctypes.c_int]
    lib.mums_shard_restart_pending.argtypes = [vp, vp]
    lib.mums_shard_stream.argtypes = [vp, vp, vp]
    lib.mums_shard_restart_plan.argtypes = [vp, vp, u32, vp, vp, vp, vp, u64, vp]
    lib.mums_shard_restart_apply.argtypes = [vp, vp, u64, vp]
    lib.mums_shard_restart_counts.argtypes = [vp, vp]
    lib.mums_shard_restart_prepare.argtypes = [vp, u32, u32, vp, vp]
    lib.mums_shard_restart_step.argtypes = [vp, vp, vp, vp]
    lib.mums_shard_restart_log.argtypes = [vp, vp, vp]
    lib.mums_shard_restart_runs.argtypes = [vp, u64, vp, vp, vp, u64, vp]
    lib.mums_shard_restart_ties.argtypes = [vp, vp, vp, u64, vp, vp]
    lib.mums_shard_restart_finish.argtypes = [vp, u64, vp, vp, vp, u64, vp, vp]
    lib.mums_shard_restart_info.argtypes = [vp, vp]
    lib.mums_shard_tie_flags.argtypes = [vp, vp, vp]
    lib.mums_shard_tie_replay.argtypes = [vp, vp, u32, u32, vp, vp, vp, vp, vp]
    lib.mums_shard_tie_apply.argtypes = [vp, vp, vp]
    lib.mums_set_match_log.argtypes = [vp, i32]
    lib.mums_set_progress_log.argtypes = [vp, i32]
    lib.mums_progress_log_copy.argtypes = [vp, ctypes.c_char_p, u64, ctypes.POINTER(u64)]
    lib.mums_match_log_copy.argtypes = [vp, vp, vp, u64, ctypes.POINTER(u64)]
    _lib = lib
    return lib


def getSeed(weight: int, seed_rank: int = 0) -> int:
    """SeedMasks.h:298-321."""
    return int(load_library().mums_get_seed(weight, seed_rank)) & 0xFFFFFFFFFFFFFFFF


def getSeedLength(seed: int) -> int:
    """SeedMasks.h:335-350."""
    if seed == 0:
        return 0
    s = seed & 0xFFFFFFFFFFFFFFFF
    lo = (s & -s).bit_length() - 1
    return s.bit_length() - lo


def getSeedWeight(seed: int) -> int:
    """SeedMasks.h:363-373."""
    return bin(seed & 0xFFFFFFFFFFFFFFFF).count("1")


def getDefaultSeedWeight(avg_len: int) -> int:
    """SeedMasks.h:389-401."""
    return int(load_library().mums_default_seed_weight(avg_len))


@dataclass
class MatchList:
    """GetMatchList output (MemHash.h:182-203): lengths[M], starts[M, G] (1-based, signed, 0 = NO_MATCH)."""

    lengths: np.ndarray
    starts: np.ndarray

    def __len__(self) -> int:
        return int(self.lengths.shape[0])

    def text(self) -> str:
        """`len\\ts0\\t...` per match (UngappedLocalAlignment.h:200-206)."""
        if len(self) == 0:
            return ""
        cols = [self.lengths.astype(np.int64)[:, None], self.starts]
        arr = np.concatenate(cols, axis=1)
        return "".join("\t".join(map(str, row)) + "\n" for row in arr.tolist())


class MemHash:
    """MemHash (MemHash.h:38) on one MI355X; genomes are added in order as in AddSequence."""

    _masked = 0

    def __init__(self, device: int = 0):
        self._lib = load_library()
        self._ctx = ctypes.c_void_p()
        rc = self._lib.mums_ctx_create(device, ctypes.byref(self._ctx))
        if rc != MUMS_OK:
            raise MumsError(rc, "mums_ctx_create failed (no HIP device? the GPU path has no CPU fallback)")
        self._seq_mask = 0
        self._keepalive: List[object] = []
        self.SetTableSize(DEFAULT_MEM_TABLE_SIZE)
        self._rt = DEFAULT_REPEAT_TOLERANCE
        self._et = DEFAULT_ENUMERATION_TOLERANCE
        self._ts = DEFAULT_MEM_TABLE_SIZE
        self._lib.mums_set_mask(self._ctx, self._masked, 0)

    # ---- lifetime ------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_ctx", None) and self._ctx.value:
            self._lib.mums_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int) -> None:
        if rc != MUMS_OK:
            msg = self._lib.mums_last_error(self._ctx).decode(errors="replace")
            if rc == MUMS_E_GAP:
                raise GapInSequence(rc, msg)
            raise MumsError(rc, msg)

    # ---- configuration (MemHash.h:72, 125-144; MaskedMemHash.h:32) ------------
    def SetTableSize(self, n: int) -> None:
        self._ts = n
        self._check(self._lib.mums_set_params(self._ctx, getattr(self, "_rt", 0), getattr(self, "_et", 1), n))

    def SetRepeatTolerance(self, t: int) -> None:
        self._rt = t
        self._check(self._lib.mums_set_params(self._ctx, t, self._et, self._ts))

    def SetEnumerationTolerance(self, t: int) -> None:
        self._et = t
        self._check(self._lib.mums_set_params(self._ctx, self._rt, t, self._ts))

    def SetSeed(self, pattern: int) -> None:
        """Seed pattern the SortedMerLists are built with (0 = default weight for the genome lengths)."""
        self._check(self._lib.mums_set_seed(self._ctx, pattern))

    # ---- input -------------------------------------------------------------------
    def AddSequence(self, seq) -> None:
        """MatchFinder::AddSequence (MatchFinder.cpp:59-87).  `seq` is bytes/str (host) or a
        torch uint8 CUDA tensor (device-resident, not copied)."""
        if hasattr(seq, "data_ptr") and getattr(seq, "is_cuda", False):
            self._keepalive.append(seq)
            self._check(self._lib.mums_add_genome_device(self._ctx, ctypes.c_void_p(seq.data_ptr()), seq.numel()))
            return
        if hasattr(seq, "data_ptr") and hasattr(seq, "is_pinned") and seq.is_contiguous() and seq.element_size() == 1:
            # a host torch uint8 tensor (e.g. pinned): copied by the library straight from its storage
            self._check(self._lib.mums_add_genome(self._ctx, ctypes.c_char_p(seq.data_ptr()) if seq.numel() else None,
                                                  seq.numel()))
            return
        if isinstance(seq, str):
            seq = seq.encode()
        b = bytes(seq)
        self._check(self._lib.mums_add_genome(self._ctx, b, len(b)))

    def Clear(self) -> None:
        """MemHash::Clear (MemHash.cpp:80-93)."""
        self._keepalive.clear()
        self._check(self._lib.mums_clear(self._ctx))

    ClearSequences = Clear

    # ---- compute -----------------------------------------------------------------
    def FindMatches(self, sequences: Optional[Sequence] = None) -> MatchList:
        """MemHash::FindMatches (MemHash.cpp:109-115): optionally AddSequence each, then find."""
        if sequences is not None:
            for s in sequences:
                self.AddSequence(s)
        self._check(self._lib.mums_find(self._ctx))
        return self.GetMatchList()

    def FindMatchesFromPosition(self, sequences: Optional[Sequence], start_points: Sequence[int]) -> MatchList:
        """MemHash::FindMatchesFromPosition (MemHash.cpp:117-127): the merge starts at SML
        index start_points[g] of every genome (FindMatchSeeds, MatchFinder.cpp:137-164)."""
        if sequences is not None:
            for s in sequences:
                self.AddSequence(s)
        sp = np.ascontiguousarray(np.asarray(start_points, dtype=np.uint64))
        self._check(self._lib.mums_set_start_points(self._ctx, sp.ctypes.data, len(sp)))
        try:
            self._check(self._lib.mums_find(self._ctx))
        finally:
            self._check(self._lib.mums_set_start_points(self._ctx, None, 0))
        return self.GetMatchList()

    def OffsetLog(self) -> np.ndarray:
        """Start points after every MER_REPEAT_LIMIT restart of the last find, one row per
        restart -- the lines MatchFinder::SetOffsetLog's stream receives (MatchFinder.cpp:152-162)."""
        rows, g = ctypes.c_uint64(), ctypes.c_uint32()
        self._check(self._lib.mums_get_offset_log(self._ctx, None, 0, ctypes.byref(rows), ctypes.byref(g)))
        out = np.zeros((int(rows.value), int(g.value)), dtype=np.uint64)
        if rows.value:
            self._check(self._lib.mums_get_offset_log(self._ctx, out.ctypes.data, rows.value, ctypes.byref(rows),
                                                      ctypes.byref(g)))
        return out

    def CreateMatches(self) -> bool:
        """MemHash::CreateMatches (MemHash.cpp:104-107)."""
        self._check(self._lib.mums_find(self._ctx))
        return True

    def SetProfiling(self, enable: bool) -> None:
        self._check(self._lib.mums_set_profiling(self._ctx, int(enable)))

    def FindStage(self, stage: int) -> None:
        self._check(self._lib.mums_find_stage(self._ctx, stage))

    def GetMatchList(self, out=None) -> MatchList:
        """MemHash::GetMatchList (MemHash.h:182-203).  out = (lengths, starts): caller-owned
        host arrays (uint64 [>= count], int64 [>= count * G], e.g. pinned memory reused across
        calls) that receive the result; the MatchList then views their first rows."""
        cnt = ctypes.c_uint64()
        g = ctypes.c_uint32()
        self._check(self._lib.mums_result_count(self._ctx, ctypes.byref(cnt), ctypes.byref(g)))
        if out is not None:
            lb, sb = out
            if lb.dtype != np.uint64 or sb.dtype != np.int64 or lb.size < cnt.value or sb.size < cnt.value * g.value \
                    or not (lb.flags.c_contiguous and sb.flags.c_contiguous):
                raise ValueError("GetMatchList(out): uint64 / int64 contiguous arrays of the result size required")
            lengths = lb.reshape(-1)[:cnt.value]
            starts = sb.reshape(-1)[:cnt.value * g.value].reshape(cnt.value, g.value)
        else:
            lengths = np.zeros(cnt.value, dtype=np.uint64)
            starts = np.zeros((cnt.value, g.value), dtype=np.int64)
        if cnt.value:
            self._check(self._lib.mums_result_copy(self._ctx, lengths.ctypes.data, starts.ctypes.data))
        return MatchList(lengths, starts)

    # ---- metrics (MemHash.h:94-105) -------------------------------------------------
    def stats(self) -> dict:
        s = _Stats()
        self._check(self._lib.mums_get_stats(self._ctx, ctypes.byref(s)))
        return {name: getattr(s, name) for name, _ in _Stats._fields_}

    def MemCount(self) -> int:
        return int(self.stats()["mem_count"])

    def MemCollisionCount(self) -> int:
        return int(self.stats()["collision_count"])

    def MemTableCount(self) -> np.ndarray:
        """MemHash::MemTableCount (MemHash.h:100): entries inserted per hash bucket."""
        T = getattr(self, "_ts", 40000)
        out = np.zeros(T, dtype=np.uint32)
        self._check(self._lib.mums_mem_table_count(self._ctx, out.ctypes.data, T))
        return out

    def PrintDistribution(self, ml: Optional["MatchList"] = None) -> str:
        """MemHash::PrintDistribution (MemHash.cpp:253-264): per bucket `i<TAB>count<TAB>bases`."""
        counts = self.MemTableCount()
        if ml is None:
            ml = self.GetMatchList()
        ends = np.cumsum(counts.astype(np.int64))
        csum = np.concatenate([[0], np.cumsum(ml.lengths.astype(np.int64))])
        bases = csum[ends] - csum[ends - counts.astype(np.int64)]
        return "".join(f"{i}\t{int(c)}\t{int(b)}\n" for i, (c, b) in enumerate(zip(counts, bases)))

    def WriteFile(self, ml: Optional["MatchList"] = None, names: Optional[Sequence[str]] = None,
                  lengths: Optional[Sequence[int]] = None) -> str:
        """MemHash::WriteFile (MemHash.cpp:301-324) text: header, then every entry bucket-major."""
        if ml is None:
            ml = self.GetMatchList()
        G = ml.starts.shape[1] if len(ml) else len(lengths or [])
        names = list(names) if names is not None else ["null"] * G
        lengths = list(lengths) if lengths is not None else [0] * G
        out = ["FormatVersion\t1\n", f"SequenceCount\t{G}\n"]
        for g in range(G):
            out.append(f"Sequence{g}File\t{names[g] or 'null'}\n")
            out.append(f"Sequence{g}Length\t{lengths[g]}\n")
        out.append(f"MatchCount\t{self.MemCount()}\n")
        out.append(ml.text())
        return "".join(out)

    def Probes(self):
        """Accepted probes of the last seed stage in AddHashEntry order: (buckets u32[P],
        ref_index u64[P]) -- hash bucket and smallest global seed-mer index of the group."""
        cnt = ctypes.c_uint64()
        self._check(self._lib.mums_probe_count(self._ctx, ctypes.byref(cnt)))
        b = np.zeros(max(cnt.value, 1), dtype=np.uint32)
        r = np.zeros(max(cnt.value, 1), dtype=np.uint64)
        self._check(self._lib.mums_probe_copy(self._ctx, b.ctypes.data, r.ctypes.data, cnt.value))
        return b[:cnt.value], r[:cnt.value]

    # ---- SortedMerList helpers (rows A3-A5) ------------------------------------------
    def SeedKeys(self, genome: int, m: int) -> np.ndarray:
        out = np.zeros(max(m, 1), dtype=np.uint64)
        self._check(self._lib.mums_copy_seed_keys(self._ctx, genome, out.ctypes.data, m))
        return out[:m]

    def SeedKeysRange(self, genome: int, first: int, count: int) -> np.ndarray:
        """GetDnaSeedMer of positions [first, first + count) of one genome."""
        out = np.zeros(count, dtype=np.uint64)
        self._check(self._lib.mums_copy_seed_keys_range(self._ctx, genome, first, count, out.ctypes.data))
        return out

    def SortedMerList(self, genome: int, m: int) -> np.ndarray:
        out = np.zeros(max(m, 1), dtype=np.uint32)
        self._check(self._lib.mums_build_sml(self._ctx, genome, out.ctypes.data, m))
        return out[:m]

    def SeedOccurrence(self, genome: int, n: int) -> np.ndarray:
        """SeedOccurrenceList::construct over genome's SML (SeedOccurrenceList.h:22-87):
        float32 getFrequency() of every position 0..n-1 (n = genome length)."""
        out = np.zeros(max(n, 1), dtype=np.float32)
        self._check(self._lib.mums_seed_occurrence(self._ctx, genome, out.ctypes.data, n))
        return out[:n]

    # ---- on-disk SortedMerList (DNAFileSML v5: FileSML.cpp:46-110, 316-374) --------------
    def WriteSML(self, genome: int, path: str, description: str = "") -> None:
        self._check(self._lib.mums_write_sml(self._ctx, genome, path.encode(), description.encode()))

    def AddSequenceFromSML(self, path: str) -> int:
        """FileSML::LoadFile: the file's sequence becomes the next genome; returns its seed."""
        seed = ctypes.c_uint64()
        self._check(self._lib.mums_add_genome_sml(self._ctx, path.encode(), ctypes.byref(seed)))
        return seed.value

    # ---- MatchList filters (MatchList.h:636-664), on the device copy of the result ----
    def MultiplicityFilter(self, mult: int) -> None:
        self._check(self._lib.mums_multiplicity_filter(self._ctx, mult))

    def LengthFilter(self, length: int) -> None:
        self._check(self._lib.mums_length_filter(self._ctx, length))

    def SetMatchLog(self, enable: bool = True) -> None:
        """MemHash::SetMatchLog (MemHash.h:149): record every inserted entry of the next FindMatches."""
        self._check(self._lib.mums_set_match_log(self._ctx, int(bool(enable))))

    def MatchLog(self) -> "MatchList":
        """The entries the match log stream received (MemHash.cpp:238-241), in insertion order."""
        n = ctypes.c_uint64()
        self._check(self._lib.mums_match_log_copy(self._ctx, None, None, 0, ctypes.byref(n)))
        g = ctypes.c_uint32()
        cnt = ctypes.c_uint64()
        self._check(self._lib.mums_result_count(self._ctx, ctypes.byref(cnt), ctypes.byref(g)))
        lengths = np.zeros(n.value, dtype=np.uint64)
        starts = np.zeros((n.value, g.value), dtype=np.int64)
        if n.value:
            self._check(self._lib.mums_match_log_copy(self._ctx, lengths.ctypes.data, starts.ctypes.data, n.value,
                                                      ctypes.byref(n)))
        return MatchList(lengths, starts)

    def LogProgress(self, enable: bool = True) -> None:
        """MatchFinder::LogProgress (MatchFinder.cpp:55-56): restate the progress text of the
        next FindMatches' merge (ProgressLog())."""
        self._check(self._lib.mums_set_progress_log(self._ctx, int(bool(enable))))

    def ProgressLog(self) -> str:
        """The text the reference's log stream receives ("N%.." per whole percent, MatchFinder.cpp:296-309)."""
        n = ctypes.c_uint64()
        self._check(self._lib.mums_progress_log_copy(self._ctx, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value + 1)
        self._check(self._lib.mums_progress_log_copy(self._ctx, buf, n.value + 1, ctypes.byref(n)))
        return buf.value.decode()

    def EliminateOverlaps(self) -> None:
        """EliminateOverlaps (Aligner.cpp:62-176) of the current MatchList, on the GPU."""
        self._check(self._lib.mums_eliminate_overlaps(self._ctx))

    def LoadMatches(self, ml: "MatchList") -> None:
        """Make a MatchList (e.g. one the caller edited) this object's current result."""
        lengths = np.ascontiguousarray(ml.lengths, dtype=np.uint64)
        starts = np.ascontiguousarray(ml.starts, dtype=np.int64)
        M, G = starts.shape
        self._check(self._lib.mums_load_matches(self._ctx, G, M, lengths.ctypes.data, starts.ctypes.data))

    def _debug_std_sort(self, keys: np.ndarray, depth: int = -1) -> np.ndarray:
        keys = np.ascontiguousarray(keys, dtype=np.uint64)
        ids = np.zeros(len(keys), dtype=np.uint32)
        self._check(self._lib.mums_debug_std_sort(self._ctx, keys.ctypes.data, len(keys), depth, ids.ctypes.data))
        return ids


def shard_key_ranges(totals, world: int):
    """The C ABI's key / bucket range cut (mums_shard_key_ranges): [(first, count)] per rank."""
    lib = load_library()
    t = np.ascontiguousarray(totals, dtype=np.uint64)
    f = np.zeros(world, dtype=np.uint32)
    c = np.zeros(world, dtype=np.uint32)
    rc = lib.mums_shard_key_ranges(t.ctypes.data, len(t), world, f.ctypes.data, c.ctypes.data)
    if rc != MUMS_OK:
        raise MumsError(rc, "mums_shard_key_ranges")
    return [(int(a), int(b)) for a, b in zip(f, c)]


class ShardedMemHash:
    """MemHash over several ranks in ONE process through the C ABI (mums_shard_run): one
    context per rank holding a contiguous genome block, one communicator per rank (RCCL
    over xGMI from mums_comm_init_all, or the host-staged in-process communicator with
    comm="local"), one host thread per rank.  The ranks' MatchLists in rank order are the
    bucket-major MatchList of MemHash::FindMatches."""

    def __init__(self, devices: Sequence[int], comm: str = "rccl", table_size: int = 40000, layout: str = "blocks",
                 parallel_compat: bool = False, chunk_size: int = 200000, pairwise: bool = False):
        """layout "blocks": a contiguous genome block per rank; "slices": every genome cut into
        world / G position slices (BASELINE config 5: two 3 Gbp genomes over 8 GPUs).
        parallel_compat: ParallelMemHash's MatchList (ParallelMemHash.cpp:42-121, CHUNK_SIZE =
        chunk_size): every rank searches a contiguous range of the chunks, the bucket owners
        re-add the ranks' tables rank after rank (compat_ranks.hip).
        pairwise: PairwiseMatchFinder's MatchList (PairwiseMatchFinder.cpp:37-73): every rank
        writes the pair rows of its key range's groups (mums_capi.hip shard_enum_rows)."""
        if layout not in ("blocks", "slices"):
            raise ValueError("layout: 'blocks' or 'slices'")
        self.layout = layout
        self.parallel_compat = bool(parallel_compat)
        self.pairwise = bool(pairwise)
        self.chunk_size = int(chunk_size)
        self._lib = load_library()
        self.devices = list(devices)
        self.world = len(self.devices)
        self.comm_kind = comm
        self.table_size = table_size
        self.seed = 0
        self.repeat_tol = 0
        self.enum_tol = 1
        self.progress = False
        self.match_log = False
        self.seqs: List[bytes] = []
        self.ranks: List[MemHash] = []
        self.stats_per_rank: List[dict] = []
        self.rank_status: List[int] = []
        comms = (ctypes.c_void_p * self.world)()
        devs = (ctypes.c_int * self.world)(*self.devices)
        init = self._lib.mums_comm_init_all if comm == "rccl" else self._lib.mums_comm_init_local
        rc = init(comms, self.world, devs)
        if rc != MUMS_OK:
            raise MumsError(rc, f"mums_comm_init ({comm}) failed")
        self._comms = [comms[r] for r in range(self.world)]

    def SetSeed(self, seed: int) -> None:
        self.seed = seed

    def SetRepeatTolerance(self, t: int) -> None:
        """MemHash::SetRepeatTolerance (MemHash.h:125-131) on every rank: the first copies of a
        genome follow its SortedMerList's std::sort order, replayed on rank g % world."""
        self.repeat_tol = int(t)

    def SetEnumerationTolerance(self, t: int) -> None:
        """MemHash::SetEnumerationTolerance (MemHash.h:137-144) on every rank: each rank
        enumerates the groups of its key range (MatchFinder.cpp:342-393, the odometer), the
        first copies in SortedMerList order (replayed like repeat tolerance)."""
        self.enum_tol = int(t)

    def LogProgress(self, enable: bool = True) -> None:
        """MatchFinder::LogProgress (MatchFinder.cpp:55-56) over the ranks: the text of the whole
        merge, restated on rank 0 (the restart is then planned on the gathered streams)."""
        self.progress = bool(enable)

    def SetMatchLog(self, enable: bool = True) -> None:
        """MemHash::SetMatchLog (MemHash.h:149; written at MemHash.cpp:238-241) under ParallelMemHash
        compat over the ranks: rank 0 restates the one-thread log with the one-context compat
        search (each chunk's thread inserts depend on every earlier chunk's entries,
        ParallelMemHash.cpp:117); MatchLog() joins the ranks' parts in rank order."""
        if enable and not self.parallel_compat:
            raise ValueError("ShardedMemHash: the match log needs parallel_compat=True")
        self.match_log = bool(enable)

    def MatchLog(self) -> MatchList:
        parts = [mh.MatchLog() for mh in self.ranks]
        G = len(self.seqs)
        if not parts:
            return MatchList(np.zeros(0, dtype=np.uint64), np.zeros((0, G), dtype=np.int64))
        return MatchList(np.concatenate([p.lengths for p in parts]),
                         np.concatenate([p.starts.reshape(-1, G) for p in parts]))

    def ProgressLog(self) -> str:
        return self.ranks[0].ProgressLog() if self.ranks else ""

    def AddSequence(self, seq) -> None:
        self.seqs.append(seq.encode() if isinstance(seq, str) else bytes(seq))

    def FindMatchesFromPosition(self, sequences: Optional[Sequence], start_points: Sequence[int],
                                stage: int = STAGE_ALL) -> MatchList:
        """MemHash::FindMatchesFromPosition (MemHash.cpp:117-127) over the ranks: every rank gets
        all G start points; the restarts are planned on the ranks' own SML parts
        (mums_shard_restart_counts .. _finish; the gathered plan as the fallback)."""
        self._start_points = np.ascontiguousarray(np.asarray(start_points, dtype=np.uint64))
        try:
            return self.FindMatches(sequences, stage)
        finally:
            self._start_points = None

    def OffsetLog(self) -> np.ndarray:
        """Start points after every MER_REPEAT_LIMIT restart of the last find (every rank holds
        the planner's log)."""
        return self.ranks[0].OffsetLog() if self.ranks else np.zeros((0, 0), dtype=np.uint64)

    def FindMatches(self, sequences: Optional[Sequence] = None, stage: int = STAGE_ALL) -> MatchList:
        import threading
        if sequences is not None:
            for s in sequences:
                self.AddSequence(s)
        G = len(self.seqs)
        lens = (ctypes.c_uint64 * G)(*[len(s) for s in self.seqs])
        base, rem = divmod(G, self.world)
        for mh in self.ranks:
            mh.close()
        self.ranks = []
        if self.layout == "slices":
            from .shard import genome_slices
            seed = self.seed or getSeed(getDefaultSeedWeight(sum(len(s) for s in self.seqs) // max(G, 1)))
            L = getSeedLength(seed)
            for r, (g, b0, b1) in enumerate(genome_slices([len(s) for s in self.seqs], L, self.world)):
                mh = MemHash(self.devices[r])
                mh.SetTableSize(self.table_size)
                mh.SetRepeatTolerance(self.repeat_tol)
                mh.SetEnumerationTolerance(self.enum_tol)
                mh.SetSeed(seed)
                mh.AddSequence(self.seqs[g][b0:min(len(self.seqs[g]), b1 + L - 1)] if b1 > b0 else b"")
                mh._check(self._lib.mums_shard_slice(mh._ctx, G, lens, g, b0, b1))
                self.ranks.append(mh)
        g0 = 0
        for r, dev in enumerate(self.devices if self.layout == "blocks" else []):
            cnt = base + (1 if r < rem else 0)
            mh = MemHash(dev)
            mh.SetTableSize(self.table_size)
            mh.SetRepeatTolerance(self.repeat_tol)
            mh.SetEnumerationTolerance(self.enum_tol)
            mh.SetSeed(self.seed)
            for s in self.seqs[g0:g0 + cnt]:
                mh.AddSequence(s)
            mh._check(self._lib.mums_shard_layout(mh._ctx, G, g0, lens))
            self.ranks.append(mh)
            g0 += cnt
        for mh in self.ranks:
            mh.LogProgress(self.progress)
            if self.parallel_compat:
                mh._check(self._lib.mums_set_parallel_compat(mh._ctx, 1, self.chunk_size))
            if self.pairwise:
                mh._check(self._lib.mums_set_pairwise(mh._ctx, 1))
            if self.match_log:
                mh.SetMatchLog(True)
        sp = getattr(self, "_start_points", None)
        if sp is not None:
            for mh in self.ranks:
                mh._check(self._lib.mums_set_start_points(mh._ctx, sp.ctypes.data, len(sp)))
        errs: List[Optional[BaseException]] = [None] * self.world
        self.rank_status = [MUMS_OK] * self.world   # every rank's mums_shard_run status

        def run(r: int) -> None:
            try:
                rc = self._lib.mums_shard_run(self.ranks[r]._ctx, self._comms[r], stage)
                self.rank_status[r] = rc
                if rc != MUMS_OK:
                    msg = self._lib.mums_last_error(self.ranks[r]._ctx).decode() or \
                        self._lib.mums_comm_last_error(self._comms[r]).decode()
                    raise MumsError(rc, f"rank {r}: {msg}")
            except BaseException as e:  # noqa: BLE001 -- reported below
                errs[r] = e

        th = [threading.Thread(target=run, args=(r,)) for r in range(self.world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for e in errs:
            if e is not None:
                raise e
        self.stats_per_rank = [mh.stats() for mh in self.ranks]
        self.restart_info = []   # per rank: path (0 none, 1 local plan, 2 gathered), candidates, restarts, bytes
        for mh in self.ranks:
            ri = np.zeros(4, dtype=np.uint64)
            mh._check(self._lib.mums_shard_restart_info(mh._ctx, ri.ctypes.data))
            self.restart_info.append({"path": int(ri[0]), "candidates": int(ri[1]), "restarts": int(ri[2]),
                                      "bytes": int(ri[3])})
        # per rank: the probes whose chains it labelled (its own key range), the chain entries
        # and the labelling's device time (mums_shard_chain_info)
        self.chain_info = []
        for mh in self.ranks:
            ci = np.zeros(4, dtype=np.uint64)
            mh._check(self._lib.mums_shard_chain_info(mh._ctx, ci.ctypes.data))
            self.chain_info.append({"probes": int(ci[0]), "chains": int(ci[1]), "ms": int(ci[2]) / 1000.0,
                                    "owned_rows": int(ci[3])})
        # per rank: what its communicator moved in the FindMatches exchange (mums_comm_exchange_info)
        self.exchange_info = []
        for c in self._comms:
            xi = np.zeros(4, dtype=np.uint64)
            if self._lib.mums_comm_exchange_info(c, xi.ctypes.data) == MUMS_OK:
                self.exchange_info.append({"sent_rows": int(xi[0]), "sent_bytes": int(xi[1]),
                                           "recv_rows": int(xi[2]), "recv_bytes": int(xi[3])})
        if stage != STAGE_ALL:
            return MatchList(np.zeros(0, dtype=np.uint64), np.zeros((0, G), dtype=np.int64))
        parts = [mh.GetMatchList() for mh in self.ranks]
        return MatchList(np.concatenate([p.lengths for p in parts]), np.concatenate([p.starts for p in parts]))

    def close(self) -> None:
        for mh in self.ranks:
            mh.close()
        self.ranks = []
        for c in self._comms:
            self._lib.mums_comm_destroy(c)
        self._comms = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def EliminateOverlaps(ml: "MatchList", device: int = 0) -> "MatchList":
    """EliminateOverlaps (Aligner.cpp:62) of a MatchList on the GPU; returns the new list."""
    with MemHash(device) as mh:
        mh.LoadMatches(ml)
        mh.EliminateOverlaps()
        return mh.GetMatchList()


class MaskedMemHash(MemHash):
    """MaskedMemHash (MaskedMemHash.h:25-40): hash only seeds whose genome-presence bitmap equals the mask."""

    _masked = 1

    def SetMask(self, seq_mask: int) -> None:
        self._seq_mask = seq_mask
        self._check(self._lib.mums_set_mask(self._ctx, 1, seq_mask))


class ParallelMemHash(MemHash):
    """ParallelMemHash (ParallelMemHash.h:29-48): the chunked OpenMP MemHash whose MatchList
    differs from MemHash's at chunk boundaries (ParallelMemHash.cpp:42-121).  The GPU
    reproduces its output (chunks cut by GetBreakpoint, searched in order, thread tables
    merged by MergeTable); chunk_size is its CHUNK_SIZE (200000, :51)."""

    CHUNK_SIZE = 200000

    def __init__(self, device: int = 0, chunk_size: int = CHUNK_SIZE):
        super().__init__(device)
        self._check(self._lib.mums_set_parallel_compat(self._ctx, 1, chunk_size))


class PairwiseMatchFinder(MemHash):
    """PairwiseMatchFinder (PairwiseMatchFinder.h:23-33): every pair of genomes that occur
    once in a seed group is hashed as a two-genome seed (PairwiseMatchFinder.cpp:37-73)."""

    def __init__(self, device: int = 0):
        super().__init__(device)
        self._check(self._lib.mums_set_pairwise(self._ctx, 1))


__all__ = [
    "MemHash", "MaskedMemHash", "ParallelMemHash", "PairwiseMatchFinder", "MatchList", "MumsError", "GapInSequence", "getSeed", "getSeedLength",
    "getSeedWeight", "getDefaultSeedWeight", "load_library", "EXPORTED_SYMBOLS", "STAGE_SEEDS", "STAGE_ALL", "ShardedMemHash",
    "shard_key_ranges", "EliminateOverlaps",
]
