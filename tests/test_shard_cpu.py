"""Sharded seed stage on CPU: gloo world_size 2 against the oracle.

The rank orchestration of libmems_amd.shard (genome blocks, balanced key ranges,
all-to-all splits, source order) runs over gloo with the CPU engine of
tests/shard_engine_cpu.py; the concatenated per-rank probe lists must equal the
oracle's AddHashEntry call sequence (bucket, first-start index) exactly.
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from libmems_amd.shard import genome_blocks, key_ranges


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_key_ranges_balanced_and_contiguous():
    rng = np.random.default_rng(1)
    tot = rng.integers(0, 1000, size=256)
    for world in (1, 2, 3, 4, 8):
        r = key_ranges(tot, world)
        assert len(r) == world
        assert r[0][0] == 0 and sum(c for _, c in r) == 256
        for (f0, c0), (f1, _) in zip(r, r[1:]):
            assert f0 + c0 == f1
        loads = [int(tot[f:f + c].sum()) for f, c in r]
        assert max(loads) - min(loads) <= 2 * int(tot.max()) + 1


def test_key_ranges_degenerate():
    assert key_ranges(np.zeros(4, np.int64), 2) == [(0, 0), (0, 4)]
    one = np.zeros(16, np.int64)
    one[5] = 100                      # every record in one bucket: one rank gets it all
    r = key_ranges(one, 4)
    assert sum(c for _, c in r) == 16
    assert sum(1 for f, c in r if one[f:f + c].sum() > 0) == 1


def test_genome_blocks():
    assert genome_blocks(8, 8) == [(g, 1) for g in range(8)]
    assert genome_blocks(8, 3) == [(0, 3), (3, 3), (6, 2)]
    assert genome_blocks(2, 4) == [(0, 1), (1, 1), (2, 0), (2, 0)]


def _worker(rank, world, port, seqs, seed, outdir):
    import torch.distributed as dist
    from libmems_amd.shard import ShardedSeedStage, genome_blocks
    from tests.shard_engine_cpu import CpuShardEngine

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        first, count = genome_blocks(len(seqs), world)[rank]
        eng = CpuShardEngine(seqs, first, count, seed)
        stage = ShardedSeedStage(eng)
        stage.run()
        b, r = eng.probes()
        np.save(os.path.join(outdir, f"b{rank}.npy"), b)
        np.save(os.path.join(outdir, f"r{rank}.npy"), r)
    finally:
        dist.destroy_process_group()


def _sharded_probes(seqs, seed, world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), seqs, seed, d), nprocs=world, join=True)
        b = np.concatenate([np.load(os.path.join(d, f"b{r}.npy")) for r in range(world)])
        r = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)])
    return b, r


@pytest.mark.parametrize("G,n,p,w,world", [(4, 60_000, 0.03, 15, 2), (3, 40_000, 0.05, 19, 2),
                                             (6, 20_000, 0.03, 19, 2)])
def test_sharded_seed_stage_matches_oracle(oracle_mod, G, n, p, w, world):
    seqs = oracle_mod.generate(G, n, p, 4242 + G)
    seed = oracle_mod.get_seed(w)
    ob, orf, st = oracle_mod.seed_probes(seqs, seed)
    assert st["probes"] > 1000
    b, r = _sharded_probes(seqs, seed, world)
    assert len(b) == len(ob)
    assert np.array_equal(b, ob)
    assert np.array_equal(r, orf)


def test_single_rank_engine_matches_oracle(oracle_mod):
    """The CPU engine alone (world 1, no process group) reproduces the oracle."""
    from libmems_amd.shard import ShardedSeedStage
    from tests.shard_engine_cpu import CpuShardEngine

    seqs = oracle_mod.generate(3, 30_000, 0.02, 99)
    seed = oracle_mod.get_seed(15)
    eng = CpuShardEngine(seqs, 0, 3, seed)
    ShardedSeedStage(eng).run()
    b, r = eng.probes()
    ob, orf, _ = oracle_mod.seed_probes(seqs, seed)
    assert np.array_equal(b, ob) and np.array_equal(r, orf)


def _find_worker(rank, world, port, seqs, seed, T, outdir):
    import torch.distributed as dist
    from libmems_amd.shard import ShardedFindMatches, genome_blocks
    from tests.shard_engine_cpu import CpuShardEngine

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        first, count = genome_blocks(len(seqs), world)[rank]
        eng = CpuShardEngine(seqs, first, count, seed, table_size=T)
        ml = ShardedFindMatches(eng).run()
        st = eng.stats()
        np.save(os.path.join(outdir, f"l{rank}.npy"), ml.lengths)
        np.save(os.path.join(outdir, f"s{rank}.npy"), ml.starts)
        np.save(os.path.join(outdir, f"c{rank}.npy"), np.array([st["mem_count"], st["collision_count"]]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("G,n,p,w,T", [(4, 60_000, 0.02, 15, 40000), (3, 50_000, 0.05, 15, 13)])
def test_sharded_find_matches_gloo_world2(oracle_mod, G, n, p, w, T):
    """Sharded FindMatches orchestration (bucket ranges, row all-to-all, packed allgather)
    under gloo world_size 2 with the CPU engine: ranks' MatchLists in rank order = the
    oracle's serial MemHash MatchList."""
    seqs = oracle_mod.generate(G, n, p, 99 + G)
    seed = oracle_mod.get_seed(w)
    ref_l, ref_s, ref_st = oracle_mod.find_matches(seqs, seed, table_size=T)
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_find_worker, args=(world, _free_port(), seqs, seed, T, d), nprocs=world, join=True)
        lens = np.concatenate([np.load(os.path.join(d, f"l{r}.npy")) for r in range(world)])
        sts = np.concatenate([np.load(os.path.join(d, f"s{r}.npy")).reshape(-1, G) for r in range(world)])
        cnt = sum(np.load(os.path.join(d, f"c{r}.npy")) for r in range(world))
    assert len(lens) == len(ref_l) > 0
    assert (lens == ref_l).all() and (sts == ref_s).all()
    assert int(cnt[0]) == ref_st["mem_count"] and int(cnt[1]) == ref_st["collision_count"]


def test_genome_slices_cover_every_position_in_order():
    """Position-sharded layout (BASELINE config 5): genome-major, position-ordered slices that
    tile every genome's SML positions exactly once (the exchange relies on rank order =
    global seed-mer index order)."""
    from libmems_amd.shard import genome_slices
    lens, L = [3_000_003, 2_000_000], 27
    sl = genome_slices(lens, L, 8)
    assert [g for g, _, _ in sl] == [0, 0, 0, 0, 1, 1, 1, 1]
    for g, n in enumerate(lens):
        parts = [(b0, b1) for gg, b0, b1 in sl if gg == g]
        assert parts[0][0] == 0 and parts[-1][1] == n - L + 1
        assert all(parts[i][1] == parts[i + 1][0] for i in range(len(parts) - 1))
        assert all(b0 % 64 == 0 for b0, _ in parts)   # packed words of a slice = the genome's
        assert all(abs((b1 - b0) - (n - L + 1) / 4) < 64 for b0, b1 in parts)
    with pytest.raises(ValueError):
        genome_slices(lens, L, 3)


def test_abi_key_ranges_match_python():
    """mums_shard_key_ranges (C ABI, host only) = shard.key_ranges for the same totals."""
    import libmems_amd as lm
    from libmems_amd.shard import key_ranges
    rng = np.random.default_rng(3)
    for nb in (1, 7, 128, 40000):
        for world in (1, 2, 3, 8):
            t = rng.integers(0, 1000, size=nb).astype(np.uint64)
            if nb > 10:
                t[rng.integers(0, nb, size=nb // 2)] = 0
            assert lm.shard_key_ranges(t, world) == key_ranges(t, world)


def _host_ops_worker(rank, world, port, outdir):
    """Calls the mums_comm_ops callbacks of host_comm_ops through their C function pointers,
    as shard_comm.hip's HostComm does, on host buffers."""
    import ctypes

    import torch.distributed as dist
    from libmems_amd.shard import host_comm_ops

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ops = host_comm_ops()
    # all-gather: rank r sends [r, r + 2^63, 7]
    send = np.array([rank, (1 << 63) + rank, 7], dtype=np.uint64)
    recv = np.zeros(3 * world, dtype=np.uint64)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    rc1 = ops.allgather_u64(None, send.ctypes.data_as(u64p), 3, recv.ctypes.data_as(u64p))
    # all-to-allv: rank r sends (p + 1) * (r + 1) bytes of value 16 r + p to peer p
    sb = np.array([(p + 1) * (rank + 1) for p in range(world)], dtype=np.uint64)
    rb = np.array([(rank + 1) * (s + 1) for s in range(world)], dtype=np.uint64)
    sbuf = np.concatenate([np.full(int(sb[p]), 16 * rank + p, dtype=np.uint8) for p in range(world)])
    rbuf = np.zeros(int(rb.sum()), dtype=np.uint8)
    rc2 = ops.alltoallv(None, sbuf.ctypes.data, sb.ctypes.data_as(u64p), rbuf.ctypes.data, rb.ctypes.data_as(u64p))
    np.save(os.path.join(outdir, f"ag{rank}.npy"), recv)
    np.save(os.path.join(outdir, f"a2a{rank}.npy"), rbuf)
    np.save(os.path.join(outdir, f"rc{rank}.npy"), np.array([rc1, rc2]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_comm_ops_gloo(world):
    """The transport mums_comm_init_host hands to mums_shard_run (shard.host_comm_ops over gloo):
    all-gather and all-to-allv blocks in rank order, exercised through the C callback types."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_host_ops_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        for r in range(world):
            assert (np.load(os.path.join(d, f"rc{r}.npy")) == 0).all()
            ag = np.load(os.path.join(d, f"ag{r}.npy"))
            exp = np.concatenate([np.array([s, (1 << 63) + s, 7], dtype=np.uint64) for s in range(world)])
            assert (ag == exp).all()
            a2a = np.load(os.path.join(d, f"a2a{r}.npy"))
            exp2 = np.concatenate([np.full((r + 1) * (s + 1), 16 * s + r, dtype=np.uint8) for s in range(world)])
            assert (a2a == exp2).all()
