"""GPU: probe order of the seed stage vs the oracle, and the sharded seed stage
 with R ranks sharing the box's GPU (exchange over gloo)."""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("G,n,p,w", [(4, 300_000, 0.02, 15), (3, 200_000, 0.05, 19), (2, 100_000, 1.0, 15)])
def test_probe_sequence_matches_oracle(gpu_lib, oracle_mod, G, n, p, w):
    """AddHashEntry call sequence (bucket, first-start index) of the GPU seed stage."""
    seqs = oracle_mod.generate(G, n, p, 4242 + G)
    seed = oracle_mod.get_seed(w)
    ob, orf, st = oracle_mod.seed_probes(seqs, seed)
    with gpu_lib.MemHash(0) as mh:
        mh.SetSeed(seed)
        for s in seqs:
            mh.AddSequence(s)
        mh.FindStage(gpu_lib.STAGE_SEEDS)
        b, r = mh.Probes()
    assert len(b) == st["probes"]
    assert np.array_equal(b, ob)
    assert np.array_equal(r, orf)


@pytest.mark.parametrize("G,n,p,w,world", [(4, 300_000, 0.02, 15, 2), (3, 200_000, 0.05, 19, 3),
                                             (6, 150_000, 0.02, 19, 2), (9, 60_000, 0.03, 15, 2)])
def test_sharded_seed_stage_gpu(oracle_mod, G, n, p, w, world):
    seqs = oracle_mod.generate(G, n, p, 4242 + G)
    ob, orf, st = oracle_mod.seed_probes(seqs, oracle_mod.get_seed(w))
    with tempfile.TemporaryDirectory() as d:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
               os.path.join(ROOT, "tests", "gpu_shard_worker.py"), d, str(G), str(n), str(p), str(w)]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        assert res.returncode == 0, res.stderr[-3000:]
        b = np.concatenate([np.load(os.path.join(d, f"b{r}.npy")) for r in range(world)])
        r = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)])
        s = [np.load(os.path.join(d, f"s{r}.npy")) for r in range(world)]
    assert sum(int(x[0]) for x in s) == st["seedmers"]
    assert np.array_equal(b, ob)
    assert np.array_equal(r, orf)


@pytest.mark.parametrize("G,n,p,w,world,ib33", [(2, 300_000, 0.02, 19, 4, False), (2, 300_000, 0.02, 19, 4, True),
                                                  (3, 200_000, 0.03, 19, 6, True), (2, 400_000, 0.01, 15, 2, False),
                                                  (2, 250_000, 0.05, 17, 8, False), (2, 300_000, 0.02, 21, 2, True),
                                                  (2, 300_000, 0.02, 21, 8, True), (3, 200_000, 0.03, 20, 6, True)])
def test_sharded_slices_gpu(oracle_mod, G, n, p, w, world, ib33):
    """Position-sharded seed stage (BASELINE config 5 layout: every genome cut into
    world/G position slices), optionally with the 33-bit records of the > 2^32 seed-mer
    case forced: the ranks' probe lists concatenated = the oracle's AddHashEntry sequence."""
    seqs = oracle_mod.generate(G, n, p, 4242 + G)
    ob, orf, st = oracle_mod.seed_probes(seqs, oracle_mod.get_seed(w))
    with tempfile.TemporaryDirectory() as d:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
               os.path.join(ROOT, "tests", "gpu_shard_worker.py"), d, str(G), str(n), str(p), str(w), "slices"]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        if ib33:
            env["MUMS_DEV_SHARD_IB33"] = "1"
        res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        assert res.returncode == 0, res.stderr[-3000:]
        b = np.concatenate([np.load(os.path.join(d, f"b{r}.npy")) for r in range(world)])
        r = np.concatenate([np.load(os.path.join(d, f"r{r}.npy")) for r in range(world)])
        s = [np.load(os.path.join(d, f"s{r}.npy")) for r in range(world)]
    assert sum(int(x[0]) for x in s) == st["seedmers"]
    assert np.array_equal(b, ob)
    assert np.array_equal(r, orf)


@pytest.mark.parametrize("G,n,p,w,world", [(2, 400_000, 0.02, 19, 2), (2, 300_000, 0.03, 19, 4)])
def test_sharded_slices_chunked_merge_gpu(oracle_mod, G, n, p, w, world):
    """A rank's key range above one onesweep merge (BASELINE config 5 on 2 or 4 GPUs: > 2^30
    records per rank) is merged in bucket chunks; forced small here (MUMS_DEV_CHUNK_RECORDS),
    with 33-bit records: the ranks' probe counts add up to the oracle's."""
    seqs = oracle_mod.generate(G, n, p, 4242 + G)
    _, _, st = oracle_mod.seed_probes(seqs, oracle_mod.get_seed(w))
    with tempfile.TemporaryDirectory() as d:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
               os.path.join(ROOT, "tests", "gpu_shard_worker.py"), d, str(G), str(n), str(p), str(w), "slices"]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", MUMS_DEV_SHARD_IB33="1",
                   MUMS_DEV_CHUNK_RECORDS=str(n // 3))
        res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        assert res.returncode == 0, res.stderr[-3000:]
        s = [np.load(os.path.join(d, f"s{r}.npy")) for r in range(world)]
    assert sum(int(x[0]) for x in s) == st["seedmers"]
    assert sum(int(x[1]) for x in s) == st["probes"]


@pytest.mark.parametrize("G,n,p,w,world,T,slices", [(4, 300_000, 0.02, 15, 2, 40000, False),
                                                      (3, 200_000, 0.05, 19, 3, 40000, False),
                                                      (5, 100_000, 1.0, 15, 2, 40000, False),
                                                      (4, 200_000, 0.01, 15, 3, 7, False),
                                                      (2, 300_000, 0.02, 19, 4, 40000, True),
                                                      (2, 200_001, 0.03, 15, 6, 7, True),
                                                      (3, 150_000, 0.02, 17, 3, 40000, True)])
def test_sharded_find_matches_gpu(oracle_mod, G, n, p, w, world, T, slices):
    """Sharded FindMatches (probe rows to bucket owners, packed-genome allgather, per-rank
    replay): the ranks' MatchLists in rank order = the oracle's MatchList, bit for bit --
    with genome blocks per rank, or position slices (BASELINE config 5 layout: the packed
    slices all-gathered into the whole genomes for the chain walks)."""
    seqs = oracle_mod.generate(G, n, p, 4242 + G)
    ref_len, ref_st, ref_stats = oracle_mod.find_matches(seqs, oracle_mod.get_seed(w), table_size=T)
    with tempfile.TemporaryDirectory() as d:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
               os.path.join(ROOT, "tests", "gpu_shard_find_worker.py"), d, str(G), str(n), str(p), str(w), str(T)]
        if slices:
            cmd.append("slices")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        assert res.returncode == 0, res.stderr[-3000:]
        lens = np.concatenate([np.load(os.path.join(d, f"len{r}.npy")) for r in range(world)])
        sts = np.concatenate([np.load(os.path.join(d, f"st{r}.npy")).reshape(-1, G) for r in range(world)])
        stats = sum(np.load(os.path.join(d, f"stats{r}.npy")) for r in range(world))
    assert len(lens) == len(ref_len)
    assert (lens == ref_len).all() and (sts == ref_st).all()
    assert int(stats[0]) == ref_stats["mem_count"] and int(stats[1]) == ref_stats["collision_count"]


@pytest.mark.parametrize("G,n,p,w,world,T,flags", [(4, 300_000, 0.02, 15, 2, 40000, ("abi",)),
                                                     (3, 200_000, 0.05, 19, 3, 7, ("abi",)),
                                                     (2, 300_000, 0.02, 19, 4, 40000, ("abi", "slices")),
                                                     (3, 200_000, 0.01, 15, 2, 40000, ("abi", "gapped")),
                                                     (2, 240_000, 0.01, 19, 4, 40000, ("abi", "slices", "gapped")),
                                                     (3, 300_000, 0.03, 15, 2, 40000, ("abi", "compat3000")),
                                                     (4, 200_000, 0.01, 15, 3, 40000, ("abi", "compat2000"))])
def test_sharded_abi_multiprocess_gpu(oracle_mod, G, n, p, w, world, T, flags):
    """mums_shard_run (the C++ orchestration of shard_comm.hip: agreement on every rank's
    status, record and row all-to-allv, packed all-gather, restart planning on rank 0) with
    ranks that are separate processes sharing cuda:0, their collectives carried by a gloo
    process group through mums_comm_init_host.  RCCL refuses two ranks on one GPU, so this
    is the multi-process path the one-GPU box can run; the ranks' MatchLists in rank order
    = the oracle's, bit for bit (N-gapped inputs: restarts planned over all ranks; "compatC":
    ParallelMemHash over the ranks)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gsfw", os.path.join(ROOT, "tests", "gpu_shard_find_worker.py"))
    gsfw = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gsfw)
    seqs = gsfw.genomes(G, n, p, flags)
    compat = [int(f[6:]) for f in flags if f.startswith("compat")]
    ref_len, ref_st, ref_stats = oracle_mod.find_matches(seqs, oracle_mod.get_seed(w), table_size=T,
                                                         parallel_compat=bool(compat),
                                                         chunk_size=compat[0] if compat else 0)
    with tempfile.TemporaryDirectory() as d:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
               os.path.join(ROOT, "tests", "gpu_shard_find_worker.py"), d, str(G), str(n), str(p), str(w), str(T),
               *flags]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        assert res.returncode == 0, res.stderr[-3000:]
        lens = np.concatenate([np.load(os.path.join(d, f"len{r}.npy")) for r in range(world)])
        sts = np.concatenate([np.load(os.path.join(d, f"st{r}.npy")).reshape(-1, G) for r in range(world)])
        stats = sum(np.load(os.path.join(d, f"stats{r}.npy")) for r in range(world))
    if "gapped" in flags:
        assert ref_stats["restarts"] > 0
    assert len(lens) == len(ref_len)
    assert (lens == ref_len).all() and (sts == ref_st).all()
    assert int(stats[0]) == ref_stats["mem_count"]
    if not compat:   # (compat: the ranks' own collisions plus the owners' re-adds)
        assert int(stats[1]) == ref_stats["collision_count"]
