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
