"""TEST INFRASTRUCTURE: a CPU engine for libmems_amd.shard.ShardedSeedStage.

Same record format and stage contract as the HIP engine (mums_shard_keys /
mums_shard_merge), restated with numpy over the oracle's seed keys, so the rank
orchestration (key ranges, all-to-all splits, source order) can run under gloo on
CPU.  Probe semantics are those of MemHash's defaults (repeat_tol 0, enum_tol 1):
EnumerateMatches (MemHash.cpp:139-162), HashMatch/SetDirection (:167-203),
CalculateOffset (MatchHashEntry.cpp:141-160), bucket (MemHash.cpp:213).
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import oracle


def ckeys(seq: bytes, seed: int, w: int) -> np.ndarray:
    """Compact canonical keys (v << 1 | parity) from the oracle's left-aligned GetDnaSeedMer keys."""
    k = oracle.seed_keys(seq, seed).astype(np.uint64)
    return ((k >> np.uint64(64 - 2 * w)) << np.uint64(1)) | (k & np.uint64(1))


class CpuShardEngine:
    def __init__(self, seqs, first: int, count: int, seed: int, table_size: int = 40000):
        self.seqs, self.first, self.count, self.seed, self.T = seqs, first, count, seed, table_size
        self.L = oracle.lib().oracle_seed_length(seed)
        self.w = bin(seed).count("1")
        self.kbits = 2 * self.w + 1
        self.B = min(11, max(self.kbits - 32, min(8, self.kbits - 1)))
        self.m = [max(len(s) - self.L + 1, 0) for s in seqs]
        self.base = np.concatenate([[0], np.cumsum(self.m)]).astype(np.int64)
        self.klow = self.kbits - self.B
        self.table_size = table_size
        self.probe_buckets = np.zeros(0, np.uint32)
        self.probe_refs = np.zeros(0, np.uint64)
        self.probe_rows_ = np.zeros((0, len(seqs) + 1), np.int64)
        self.result = None

    def msd_bits(self):
        return self.B, int(sum(self.m[self.first:self.first + self.count]))

    def alloc(self, n: int) -> torch.Tensor:
        return torch.empty(max(n, 1), dtype=torch.int64)

    def keys(self, rec: torch.Tensor, nb: int) -> np.ndarray:
        parts_k, parts_i = [], []
        for g in range(self.first, self.first + self.count):
            parts_k.append(ckeys(self.seqs[g], self.seed, self.w))
            parts_i.append(np.arange(self.m[g], dtype=np.uint64) + np.uint64(self.base[g]))
        ck = np.concatenate(parts_k) if parts_k else np.zeros(0, np.uint64)
        gi = np.concatenate(parts_i) if parts_i else np.zeros(0, np.uint64)
        bucket = (ck >> np.uint64(self.klow)).astype(np.int64)
        r = ((ck & np.uint64((1 << self.klow) - 1)) << np.uint64(32)) | gi
        order = np.argsort(bucket, kind="stable")
        if r.size:
            rec[:r.size] = torch.from_numpy(r[order].view(np.int64))
        return np.bincount(bucket, minlength=nb).astype(np.uint64)

    def merge(self, recv: torch.Tensor, nsrc: int, first: int, nbuckets: int, counts: np.ndarray) -> None:
        counts = np.asarray(counts, dtype=np.int64).reshape(nsrc, nbuckets)
        n = int(counts.sum())
        src = recv[:n].numpy().view(np.uint64)
        # source-major -> bucket-major (sources in rank order inside each bucket)
        src_off = np.concatenate([[0], np.cumsum(counts.sum(axis=1))])
        pieces, bidx = [], []
        for b in range(nbuckets):
            for s in range(nsrc):
                o = src_off[s] + counts[s, :b].sum()
                pieces.append(src[o:o + counts[s, b]])
                bidx.append(np.full(counts[s, b], first + b, dtype=np.uint64))
        r = np.concatenate(pieces) if pieces else np.zeros(0, np.uint64)
        bk = np.concatenate(bidx) if bidx else np.zeros(0, np.uint64)
        ck = (bk << np.uint64(self.klow)) | (r >> np.uint64(32))
        gi = (r & np.uint64(0xFFFFFFFF)).astype(np.int64)
        order = np.argsort(ck, kind="stable")       # stable: equal keys keep global-index order
        ck, gi = ck[order], gi[order]
        gk = ck >> np.uint64(1)
        par = (ck & np.uint64(1)).astype(np.int64)
        G = len(self.seqs)
        heads = np.flatnonzero(np.concatenate([[True], gk[1:] != gk[:-1]])) if ck.size else np.zeros(0, int)
        ends = np.concatenate([heads[1:], [ck.size]]).astype(int)
        pb, pr, rows = [], [], []
        T = self.T
        for h, e in zip(heads, ends):
            if e - h < 2 or e - h > G:
                continue
            idx = gi[h:e]
            gen = np.searchsorted(self.base, idx, side="right") - 1
            if len(set(gen.tolist())) != e - h:
                continue
            k = int(np.argmin(gen))
            sref = int(idx[k] - self.base[gen[k]]) + 1
            pref = int(par[h + k])
            off = 0
            for j in range(e - h):
                if j == k:
                    continue
                s = int(idx[j] - self.base[gen[j]]) + 1
                off += (-s - sref - self.L) if int(par[h + j]) != pref else (s - sref)
            pb.append(((off % T) + T) % T)
            pr.append(int(idx.min()))
            row = np.zeros(G + 1, np.int64)   # SetDirection (MemHash.cpp:189-203) + CalculateOffset
            for j in range(e - h):
                s = int(idx[j] - self.base[gen[j]]) + 1
                row[gen[j]] = -s if (j != k and int(par[h + j]) != pref) else s
            row[G] = off
            rows.append(row)
        self.probe_buckets = np.array(pb, dtype=np.uint32)
        self.probe_refs = np.array(pr, dtype=np.uint64)
        self.probe_rows_ = np.array(rows, dtype=np.int64).reshape(-1, G + 1)

    def probes(self):
        return self.probe_buckets, self.probe_refs

    # ---- sharded FindMatches contract (mums_shard_bucket_counts / probe_rows / packed / find)
    def bucket_counts(self) -> np.ndarray:
        return np.bincount(self.probe_buckets, minlength=self.T).astype(np.uint64)

    def probe_rows(self, bounds):
        dest = np.searchsorted(np.asarray(bounds), self.probe_buckets, side="right") - 1
        order = np.argsort(dest, kind="stable")
        counts = np.bincount(dest, minlength=len(bounds) - 1).astype(np.uint64)
        return torch.from_numpy(np.ascontiguousarray(self.probe_rows_[order])), counts

    def packed(self):
        return 0, torch.zeros(0, dtype=torch.int32), 0   # the oracle replay reads the sequences

    def find(self, rows: torch.Tensor, packed_all: torch.Tensor) -> None:
        self.result = oracle.replay_rows(self.seqs, self.seed, rows.numpy(), self.T)

    def matches(self):
        class _ML:
            pass
        ml = _ML()
        ml.lengths, ml.starts = self.result[0], self.result[1]
        return ml

    def stats(self) -> dict:
        return dict(self.result[2]) if self.result else {}
