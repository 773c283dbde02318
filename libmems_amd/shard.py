"""Sharded MemHash seed stage across GPUs: genome-per-rank keys,
key-range exchange, per-rank merge of one key range.

The reference builds one SortedMerList per genome (MemorySML::Create,
MemorySML.cpp:45-60) and merges all G of them in masked-key order in one thread
(MatchFinder::SearchRange, MatchFinder.cpp:172-340) before MemHash accepts each
key group (MemHash::EnumerateMatches, MemHash.cpp:139-162).  Here every rank owns a
contiguous block of genomes (one process per GPU):

  1. keys    : the rank's genomes -> 8-B records (ckey_low << 32 | global index),
               stably bucketed by the top B key bits (HIP, mums_shard_keys);
  2. ranges  : per-bucket counts all-gathered; the 2^B buckets are cut into
               world_size contiguous key ranges of balanced record counts;
  3. exchange: one all-to-all (RCCL over xGMI on GPUs) sends every bucket range to
               its owner; sources arrive in rank order = global index order;
  4. merge   : each rank sorts / groups / accepts its key range (mums_shard_merge).

Rank r's probes are the reference's AddHashEntry calls for the keys of range r, so
concatenating the ranks' probe lists in rank order reproduces the single-process
order exactly.  The engine is pluggable: HipShardEngine drives the C ABI; tests
drive the same orchestration with a CPU engine over gloo.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import MemHash


def key_ranges(bucket_totals: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Cut buckets [0, nb) into `world` contiguous ranges (first, count) whose record
    totals are as even as bucket granularity allows (boundary r at the first bucket whose
    prefix sum reaches r/world of the total).  Deterministic from the totals alone, so
    every rank computes the same cut."""
    nb = int(bucket_totals.shape[0])
    cum = np.concatenate([[0], np.cumsum(bucket_totals.astype(np.int64))])
    total = int(cum[-1])
    bounds = [0]
    for r in range(1, world):
        target = (total * r + world - 1) // world
        b = int(np.searchsorted(cum, target, side="left"))
        bounds.append(min(max(b, bounds[-1]), nb))
    bounds.append(nb)
    return [(bounds[r], bounds[r + 1] - bounds[r]) for r in range(world)]


def genome_blocks(G: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous genome block (first, count) per rank; earlier ranks take the remainder."""
    base, rem = divmod(G, world)
    out, g = [], 0
    for r in range(world):
        c = base + (1 if r < rem else 0)
        out.append((g, c))
        g += c
    return out


def genome_slices(lengths: Sequence[int], L: int, world: int) -> List[Tuple[int, int, int]]:
    """Position-sharded layout (BASELINE config 5: each 3 Gbp genome over world/G ranks):
    rank r owns SML positions [begin, end) of genome g = r // (world / G), the genome's
    SMLLength cut into world / G near-equal ranges whose inner bounds fall on 64-base
    boundaries (a slice's 2-bit packed words are then exactly the genome's words for its
    bases: the FindMatches all-gather of the packed genomes).  Rank order = genome-major,
    position order = global seed-mer index order, as the exchange requires."""
    G = len(lengths)
    if G == 0 or world % G:
        raise ValueError("position sharding needs world_size to be a multiple of the genome count")
    k = world // G
    out = []
    for g, n in enumerate(lengths):
        m = max(int(n) - L + 1, 0)
        cut = [0] + [(m * j // k) // 64 * 64 for j in range(1, k)] + [m]
        for j in range(k):
            out.append((g, cut[j], max(cut[j], cut[j + 1])))
    return out


class HipShardEngine:
    """One rank's MemHash context in sharded mode (C ABI, HIP kernels on `device`).
    slice_of = (genome, begin, end): position-sharded layout (genome_slices); `genomes`
    is then the one ASCII slice holding bases [begin, end + L - 1) of that genome."""

    def __init__(self, device: int, seed: int, lengths: Sequence[int], first: int, genomes: Sequence,
                 profiling: bool = False, table_size: int = 40000,
                 slice_of: Optional[Tuple[int, int, int]] = None):
        self.mh = MemHash(device)
        self.device = torch.device("cuda", device)
        self.G = len(lengths)
        self.table_size = int(table_size)
        self.mh.SetTableSize(self.table_size)
        self.mh.SetSeed(seed)
        for s in genomes:
            self.mh.AddSequence(s)
        lens = (ctypes.c_uint64 * len(lengths))(*[int(x) for x in lengths])
        lib = self.mh._lib
        if slice_of is None:
            self.mh._check(lib.mums_shard_layout(self.mh._ctx, len(lengths), first, lens))
        else:
            g, b0, b1 = slice_of
            self.mh._check(lib.mums_shard_slice(self.mh._ctx, len(lengths), lens, g, b0, b1))
        if profiling:
            self.mh.SetProfiling(True)

    def msd_bits(self) -> Tuple[int, int]:
        b, n = ctypes.c_uint32(), ctypes.c_uint64()
        self.mh._check(self.mh._lib.mums_shard_msd_bits(self.mh._ctx, ctypes.byref(b), ctypes.byref(n)))
        return int(b.value), int(n.value)

    def alloc(self, n: int) -> torch.Tensor:
        return torch.empty(max(n, 1), dtype=torch.int64, device=self.device)

    def keys(self, rec: torch.Tensor, nb: int) -> np.ndarray:
        counts = np.zeros(nb, dtype=np.uint64)
        self.mh._check(self.mh._lib.mums_shard_keys(self.mh._ctx, ctypes.c_void_p(rec.data_ptr()), rec.numel(),
                                                     counts.ctypes.data))
        return counts

    def merge(self, recv: torch.Tensor, nsrc: int, first: int, nbuckets: int, counts: np.ndarray) -> None:
        c = np.ascontiguousarray(counts, dtype=np.uint64)
        self.mh._check(self.mh._lib.mums_shard_merge(self.mh._ctx, ctypes.c_void_p(recv.data_ptr()), nsrc, first,
                                                      nbuckets, c.ctypes.data))

    def stats(self) -> dict:
        return self.mh.stats()

    def probes(self):
        return self.mh.Probes()

    # ---- sharded FindMatches (mums_shard_bucket_counts / probe_rows / packed / find)
    def bucket_counts(self) -> np.ndarray:
        c = np.zeros(self.table_size, dtype=np.uint64)
        self.mh._check(self.mh._lib.mums_shard_bucket_counts(self.mh._ctx, c.ctypes.data))
        return c

    def probe_rows(self, bounds: Sequence[int]) -> Tuple[torch.Tensor, np.ndarray]:
        n = ctypes.c_uint64()
        self.mh._check(self.mh._lib.mums_probe_count(self.mh._ctx, ctypes.byref(n)))
        rows = torch.empty((max(n.value, 1), self.G + 1), dtype=torch.int64, device=self.device)
        b = np.ascontiguousarray(bounds, dtype=np.uint32)
        counts = np.zeros(len(bounds) - 1, dtype=np.uint64)
        self.mh._check(self.mh._lib.mums_shard_probe_rows(self.mh._ctx, len(bounds) - 1, b.ctypes.data,
                                                           ctypes.c_void_p(rows.data_ptr()), rows.shape[0],
                                                           counts.ctypes.data))
        return rows[:n.value], counts

    def packed(self) -> Tuple[int, torch.Tensor, int]:
        off, n, tot = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        self.mh._check(self.mh._lib.mums_shard_packed_info(self.mh._ctx, ctypes.byref(off), ctypes.byref(n),
                                                            ctypes.byref(tot)))
        words = torch.empty(max(n.value, 1), dtype=torch.int32, device=self.device)
        self.mh._check(self.mh._lib.mums_shard_packed_copy(self.mh._ctx, ctypes.c_void_p(words.data_ptr())))
        return int(off.value), words[:n.value], int(tot.value)

    def find(self, rows: torch.Tensor, packed_all: torch.Tensor) -> None:
        rows = rows.to(self.device).contiguous()
        packed_all = packed_all.to(self.device).contiguous()
        torch.cuda.synchronize(self.device)
        self.mh._check(self.mh._lib.mums_shard_find(self.mh._ctx, ctypes.c_void_p(rows.data_ptr()), rows.shape[0],
                                                     ctypes.c_void_p(packed_all.data_ptr())))

    def matches(self):
        return self.mh.GetMatchList()

    def close(self) -> None:
        self.mh.close()


class ShardedSeedStage:
    """Orchestrates steps 1-4 for one rank of the default process group (or `group`)."""

    def __init__(self, engine, group: Optional[dist.ProcessGroup] = None):
        self.engine = engine
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        backend = dist.get_backend(group) if dist.is_initialized() else "none"
        # collectives run where the backend wants their tensors: RCCL on the GPU, gloo on the host
        self.wire = "cuda" if backend == "nccl" else "cpu"
        self.last_range: Tuple[int, int] = (0, 0)
        self.last_exchange_bytes = 0

    def _all_gather_counts(self, counts: np.ndarray) -> np.ndarray:
        if self.world == 1:
            return counts[None, :].astype(np.int64)
        t = torch.from_numpy(counts.astype(np.int64)).to(self.wire)
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        return torch.stack(parts).cpu().numpy()

    def run_find(self) -> None:
        """Steps 1-8 (ShardedFindMatches over the same process group)."""
        if getattr(self, "_find", None) is None:
            self._find = ShardedFindMatches(self.engine, self.group)
        self._find.run()

    def run(self) -> None:
        eng = self.engine
        B, n_local = eng.msd_bits()
        nb = 1 << B
        rec = eng.alloc(n_local)
        counts = eng.keys(rec, nb)
        C = self._all_gather_counts(counts)                 # [world, nb]
        ranges = key_ranges(C.sum(axis=0), self.world)
        first, cnt = ranges[self.rank]
        self.last_range = (first, cnt)
        sub = np.ascontiguousarray(C[:, first:first + cnt])
        if self.world == 1:
            eng.merge(rec, 1, first, cnt, sub)
            return
        send = [int(C[self.rank, f:f + c].sum()) for f, c in ranges]
        recv = [int(C[s, first:first + cnt].sum()) for s in range(self.world)]
        src = rec[:n_local] if n_local else rec[:0]
        if self.wire == "cpu" and src.is_cuda:
            src = src.cpu()
        out = torch.empty(sum(recv), dtype=torch.int64, device=src.device)
        dist.all_to_all_single(out, src.contiguous(), recv, send, group=self.group)
        if self.wire == "cuda":
            torch.cuda.current_stream().synchronize()     # the engine runs on its own stream
        self.last_exchange_bytes = 8 * (sum(send) - send[self.rank])
        if out.device != rec.device:
            out = out.to(rec.device)
            if out.is_cuda:
                torch.cuda.current_stream().synchronize()
        eng.merge(out, self.world, first, cnt, sub)


class ShardedFindMatches:
    """Sharded MemHash::FindMatches for one rank: the sharded seed
    stage, then the probes move to the rank owning their hash bucket and every rank
    replays its bucket range (chain labelling + AddHashEntry, MemHash.cpp:209-251):

      5. buckets : per-bucket probe counts all-gathered; the hash buckets are cut into
                   world_size contiguous ranges of balanced probe counts;
      6. rows    : every probe as G+1 int64 {starts, offset}, grouped by owner rank in
                   key order; one all-to-all (sources in rank order = key order);
      7. genomes : every rank's 2-bit packed genomes all-gathered (chain walks read any
                   genome);
      8. find    : chain labelling + replay of the rank's buckets (mums_shard_find).

    The ranks' MatchLists concatenated in rank order are the reference's bucket-major
    MatchList (MemHash.h:182-203)."""

    def __init__(self, engine, group: Optional[dist.ProcessGroup] = None):
        self.engine = engine
        self.group = group
        self.seeds = ShardedSeedStage(engine, group)
        self.world, self.rank, self.wire = self.seeds.world, self.seeds.rank, self.seeds.wire
        self.bucket_range: Tuple[int, int] = (0, 0)
        self.last_exchange_bytes = 0

    def _gather_np(self, a: np.ndarray) -> np.ndarray:
        return self.seeds._all_gather_counts(a)

    def run(self):
        eng = self.engine
        self.seeds.run()
        T = eng.table_size
        C = self._gather_np(eng.bucket_counts())                     # [world, T]
        ranges = key_ranges(C.sum(axis=0), self.world)
        bounds = [f for f, _ in ranges] + [T]
        self.bucket_range = ranges[self.rank]
        rows, send = eng.probe_rows(bounds)                           # [P, G+1], per-destination counts
        W = rows.shape[1]
        S = self._gather_np(send.astype(np.int64))                    # [src, dst]
        recv = [int(S[s, self.rank]) for s in range(self.world)]
        if self.world == 1:
            recv_rows = rows
        else:
            src = rows if self.wire == "cuda" else rows.cpu()
            out = torch.empty((sum(recv), W), dtype=torch.int64, device=src.device)
            dist.all_to_all_single(out.view(-1), src.contiguous().view(-1), [r * W for r in recv],
                                   [int(c) * W for c in send], group=self.group)
            if self.wire == "cuda":
                torch.cuda.current_stream().synchronize()
            self.last_exchange_bytes = 8 * W * (int(send.sum()) - int(send[self.rank]))
            recv_rows = out
        off, words, total = eng.packed()
        full = self._all_gather_packed(off, words, total)
        eng.find(recv_rows, full)
        return eng.matches()

    def _all_gather_packed(self, off: int, words: torch.Tensor, total: int) -> torch.Tensor:
        if self.world == 1:
            full = torch.zeros(total, dtype=torch.int32, device=words.device)
            full[off:off + words.numel()] = words
            return full
        meta = self._gather_np(np.array([off, words.numel()], dtype=np.int64))
        mx = int(meta[:, 1].max())
        dev = words.device if self.wire == "cuda" else torch.device("cpu")
        pad = torch.zeros(max(mx, 1), dtype=torch.int32, device=dev)
        pad[:words.numel()] = words.to(dev)
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(parts, pad, group=self.group)
        full = torch.zeros(total, dtype=torch.int32, device=dev)
        for r in range(self.world):
            o, n = int(meta[r, 0]), int(meta[r, 1])
            full[o:o + n] = parts[r][:n]
        return full


def host_comm_ops(group: Optional[dist.ProcessGroup] = None):
    """mums_comm_ops over torch.distributed on host tensors (gloo): the C ABI stages device
    data through host memory and calls these for its all-gather and all-to-allv.  Returns
    the ops struct (keep it alive as long as the communicator)."""
    import libmems_amd as lm

    world = dist.get_world_size(group)

    def allgather(_user, send, n, recv):
        try:
            src = torch.from_numpy(np.ctypeslib.as_array(send, shape=(n,)).astype(np.int64))
            outs = [torch.empty(n, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(outs, src, group=group)
            dst = np.ctypeslib.as_array(recv, shape=(world * n,))
            for r in range(world):
                dst[r * n:(r + 1) * n] = outs[r].numpy().view(np.uint64)
            return 0
        except Exception:   # a failed collective is reported through the status code
            return 1

    def alltoallv(_user, send, send_bytes, recv, recv_bytes):
        try:
            sb = [int(send_bytes[p]) for p in range(world)]
            rb = [int(recv_bytes[p]) for p in range(world)]
            src = torch.frombuffer((ctypes.c_char * max(sum(sb), 1)).from_address(send), dtype=torch.uint8)[:sum(sb)]
            out = torch.empty(sum(rb), dtype=torch.uint8)
            dist.all_to_all_single(out, src.clone(), rb, sb, group=group)
            if sum(rb):
                ctypes.memmove(recv, out.data_ptr(), sum(rb))
            return 0
        except Exception:
            return 1

    return lm.MumsCommOps(lm.COMM_ALLGATHER_FN(allgather), lm.COMM_ALLTOALLV_FN(alltoallv))


class AbiShardStage:
    """The sharded pipeline of one rank run by the C ABI itself (mums_shard_run,
    shard_comm.hip).  comm="rccl": RCCL communicator from ncclCommInitRank, its unique id
    broadcast over the default process group (any backend: only the 128-byte id and the
    control travel there); comm="host": the process group itself carries the collectives
    (mums_comm_init_host with host_comm_ops, e.g. gloo; ranks may share one GPU).
    stage = STAGE_SEEDS (steps 1-4) or STAGE_ALL (1-8)."""

    def __init__(self, engine, device: int, stage: int = 1, group: Optional[dist.ProcessGroup] = None,
                 comm: str = "rccl"):
        self.engine = engine
        self.stage = stage
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        lib = engine.mh._lib
        self.last_exchange_bytes = 0
        if comm == "host":
            self._ops = host_comm_ops(group)
            self.comm = ctypes.c_void_p()
            rc = lib.mums_comm_init_host(ctypes.byref(self.comm), device, self.world, self.rank,
                                         ctypes.byref(self._ops), None)
            if rc != 0:
                raise RuntimeError(f"mums_comm_init_host failed ({rc})")
            return
        uid = ctypes.create_string_buffer(128)
        if self.rank == 0:
            engine.mh._check(lib.mums_comm_unique_id(uid, 128))
        obj = [bytes(uid.raw)]
        if self.world > 1:
            dist.broadcast_object_list(obj, src=0, group=group)
        self.comm = ctypes.c_void_p()
        rc = lib.mums_comm_init_rank(ctypes.byref(self.comm), device, self.world, self.rank, obj[0])
        if rc != 0:
            raise RuntimeError(f"mums_comm_init_rank failed ({rc})")
        self.last_exchange_bytes = 0

    def run(self) -> None:
        lib = self.engine.mh._lib
        rc = lib.mums_shard_run(self.engine.mh._ctx, self.comm, self.stage)
        if rc != 0:
            raise RuntimeError(f"mums_shard_run: {lib.mums_last_error(self.engine.mh._ctx).decode()} / "
                               f"{lib.mums_comm_last_error(self.comm).decode()}")

    def run_find(self) -> None:
        """The whole sharded FindMatches (steps 1-8): this rank's buckets of the MatchList."""
        lib = self.engine.mh._lib
        rc = lib.mums_shard_run(self.engine.mh._ctx, self.comm, 2)   # MUMS_STAGE_ALL
        if rc != 0:
            raise RuntimeError(f"mums_shard_run: {lib.mums_last_error(self.engine.mh._ctx).decode()} / "
                               f"{lib.mums_comm_last_error(self.comm).decode()}")

    def chain_info(self) -> dict:
        """This rank's share of the last sharded FindMatches' chain stage (mums_shard_chain_info):
        the probes whose chains it labelled (its own key range), the chain entries, the time."""
        import numpy as np
        ci = np.zeros(4, dtype=np.uint64)
        self.engine.mh._check(self.engine.mh._lib.mums_shard_chain_info(self.engine.mh._ctx, ci.ctypes.data))
        xi = np.zeros(4, dtype=np.uint64)
        self.engine.mh._lib.mums_comm_exchange_info(self.comm, xi.ctypes.data)
        return {"probes": int(ci[0]), "chains": int(ci[1]), "ms": int(ci[2]) / 1000.0, "owned_rows": int(ci[3]),
                "sent_rows": int(xi[0]), "sent_bytes": int(xi[1]), "recv_rows": int(xi[2]), "recv_bytes": int(xi[3])}

    def close(self) -> None:
        if self.comm:
            self.engine.mh._lib.mums_comm_destroy(self.comm)
            self.comm = ctypes.c_void_p()


__all__ = ["key_ranges", "genome_blocks", "HipShardEngine", "ShardedSeedStage", "ShardedFindMatches", "AbiShardStage",
           "host_comm_ops"]
