"""TEST INFRASTRUCTURE: one rank of the sharded seed stage on the HIP engine.

Launched by tests/test_gpu_shard.py as
    python -m torch.distributed.run --nproc-per-node R ... tests/gpu_shard_worker.py OUTDIR G n p w [slices]
Every rank runs its genome block (or, with "slices", its genome position slice) on cuda:0
(the test box has one GPU; the exchange goes over gloo on the host) and saves its probe list.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from libmems_amd.shard import HipShardEngine, ShardedSeedStage, genome_blocks, genome_slices  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    outdir, G, n, p, w = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]), int(sys.argv[5])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    seqs = oracle.generate(G, n, p, 4242 + G)
    seed = oracle.get_seed(w)
    dev = torch.device("cuda", 0)
    lens = [len(s) for s in seqs]
    if len(sys.argv) > 6 and sys.argv[6] == "slices":
        L = oracle.lib().oracle_seed_length(seed)
        g, b0, b1 = genome_slices(lens, L, world)[rank]
        part = seqs[g][b0:min(lens[g], b1 + L - 1)] if b1 > b0 else b""
        local = [torch.frombuffer(bytearray(part), dtype=torch.uint8).to(dev)] if part else \
            [torch.zeros(0, dtype=torch.uint8, device=dev)]
        eng = HipShardEngine(0, seed, lens, g, local, slice_of=(g, b0, b1))
    else:
        first, count = genome_blocks(G, world)[rank]
        local = [torch.frombuffer(bytearray(s), dtype=torch.uint8).to(dev) for s in seqs[first:first + count]]
        eng = HipShardEngine(0, seed, lens, first, local)
    ShardedSeedStage(eng).run()
    st = eng.stats()
    if os.environ.get("MUMS_DEV_CHUNK_RECORDS"):   # chunked merge: counts only (no probe export)
        b, r = np.zeros(0, dtype=np.uint32), np.zeros(0, dtype=np.uint64)
    else:
        b, r = eng.probes()
    np.save(os.path.join(outdir, f"b{rank}.npy"), b)
    np.save(os.path.join(outdir, f"r{rank}.npy"), r)
    np.save(os.path.join(outdir, f"s{rank}.npy"), np.array([st["seedmers"], st["probes"], st["groups"]]))
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
