"""TEST INFRASTRUCTURE: one rank of the sharded FindMatches on the HIP engine.

Launched by tests/test_gpu_shard.py as
    python -m torch.distributed.run --nproc-per-node R ... tests/gpu_shard_find_worker.py OUTDIR G n p w T [slices]
Every rank runs its genome block (or, with "slices", its genome position slice) on cuda:0
(one GPU on the test box; exchanges over gloo) and saves its part of the MatchList (its
hash-bucket range, bucket-major).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from libmems_amd.shard import HipShardEngine, ShardedFindMatches, genome_blocks, genome_slices  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    outdir, G, n, p, w, T = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]), int(sys.argv[5]),
                             int(sys.argv[6]))
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    seqs = oracle.generate(G, n, p, 4242 + G)
    seed = oracle.get_seed(w)
    dev = torch.device("cuda", 0)
    lens = [len(s) for s in seqs]
    if len(sys.argv) > 7 and sys.argv[7] == "slices":
        L = oracle.lib().oracle_seed_length(seed)
        g, b0, b1 = genome_slices(lens, L, world)[rank]
        part = seqs[g][b0:min(lens[g], b1 + L - 1)] if b1 > b0 else b""
        local = [torch.frombuffer(bytearray(part), dtype=torch.uint8).to(dev)] if part else \
            [torch.zeros(0, dtype=torch.uint8, device=dev)]
        eng = HipShardEngine(0, seed, lens, g, local, table_size=T, slice_of=(g, b0, b1))
    else:
        first, count = genome_blocks(G, world)[rank]
        local = [torch.frombuffer(bytearray(s), dtype=torch.uint8).to(dev) for s in seqs[first:first + count]]
        eng = HipShardEngine(0, seed, lens, first, local, table_size=T)
    ml = ShardedFindMatches(eng).run()
    st = eng.stats()
    np.save(os.path.join(outdir, f"len{rank}.npy"), ml.lengths)
    np.save(os.path.join(outdir, f"st{rank}.npy"), ml.starts)
    np.save(os.path.join(outdir, f"stats{rank}.npy"), np.array([st["mem_count"], st["collision_count"]]))
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
