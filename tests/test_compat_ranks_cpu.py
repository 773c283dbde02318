"""ParallelMemHash compat over ranks on CPU (the GPU path is
shard_comm.hip compat_shard_run + compat_ranks.hip): the oracle's per-rank tables (chunk
ranges from empty tables) re-added rank after rank give the one-thread MatchList, directly
and through the exchange compat_shard_run makes (per-bucket counts all-gathered, balanced
bucket ranges, an all-to-all of the table rows, the owners' merge in source order) under
gloo world_size 2."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from libmems_amd.shard import key_ranges


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("G,n,p,w,chunk,gseed", [(3, 300_000, 0.03, 15, 3000, 2), (4, 200_000, 0.01, 15, 2000, 3),
                                                 (3, 200_000, 1.0, 11, 1003, 6)])
@pytest.mark.parametrize("ranks", [2, 3, 5])
def test_rank_tables_merge_to_one_thread(oracle_mod, G, n, p, w, chunk, gseed, ranks):
    seqs = oracle_mod.generate(G, n, p, gseed)
    seed = oracle_mod.get_seed(w)
    l1, s1, x1 = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk)
    tabs = []
    for r in range(ranks):
        l, s, _ = oracle_mod.compat_rank_table(seqs, seed, chunk, r, ranks)
        b = oracle_mod.entry_buckets(l, s)
        assert (np.diff(b) >= 0).all()   # a table in bucket order
        tabs.append((l, s))
    assert x1["chunks"] > ranks
    lm, sm, _ = oracle_mod.merge_tables(tabs, G)
    assert np.array_equal(lm, l1) and np.array_equal(sm, s1)


def _worker(rank, world, port, seqs, seed, chunk, T, outdir):
    import torch
    import torch.distributed as dist
    from oracle import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G = len(seqs)
        l, s, _ = oracle.compat_rank_table(seqs, seed, chunk, rank, world, table_size=T)
        counts = np.bincount(oracle.entry_buckets(l, s, T), minlength=T).astype(np.int64)
        allc = [torch.zeros(T, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allc, torch.from_numpy(counts))
        C = np.stack([c.numpy() for c in allc])             # [world, T]
        ranges = key_ranges(C.sum(axis=0), world)
        f, c = ranges[rank]
        rows = np.concatenate([l.astype(np.int64)[:, None], s], axis=1) if len(l) else np.zeros((0, G + 1), np.int64)
        send = [int(counts[f0:f0 + c0].sum()) for f0, c0 in ranges]          # rows per owner (bucket order)
        recv = [int(C[s2, f:f + c].sum()) for s2 in range(world)]           # rows per source
        out = torch.zeros(sum(recv) * (G + 1), dtype=torch.int64)
        dist.all_to_all_single(out, torch.from_numpy(np.ascontiguousarray(rows).reshape(-1)),
                               [x * (G + 1) for x in recv], [x * (G + 1) for x in send])
        got = out.numpy().reshape(-1, G + 1)
        srcs, o = [], 0
        for x in recv:   # the owner re-adds the sources' tables in rank order
            srcs.append((got[o:o + x, 0].astype(np.uint64), got[o:o + x, 1:]))
            o += x
        ml, ms, _ = oracle.merge_tables(srcs, G, T)
        np.save(os.path.join(outdir, f"l{rank}.npy"), ml)
        np.save(os.path.join(outdir, f"s{rank}.npy"), ms)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("G,n,p,w,chunk,T", [(3, 300_000, 0.03, 15, 3000, 40000), (4, 200_000, 0.02, 15, 2500, 7)])
def test_compat_ranks_gloo_world2(oracle_mod, G, n, p, w, chunk, T):
    seqs = oracle_mod.generate(G, n, p, 31 + G)
    seed = oracle_mod.get_seed(w)
    l1, s1, _ = oracle_mod.find_matches(seqs, seed, parallel_compat=True, chunk_size=chunk, table_size=T)
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), seqs, seed, chunk, T, d), nprocs=world, join=True)
        lens = np.concatenate([np.load(os.path.join(d, f"l{r}.npy")) for r in range(world)])
        sts = np.concatenate([np.load(os.path.join(d, f"s{r}.npy")).reshape(-1, G) for r in range(world)])
    assert np.array_equal(lens, l1) and np.array_equal(sts, s1)
