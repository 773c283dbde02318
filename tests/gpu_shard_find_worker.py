"""TEST INFRASTRUCTURE: one rank of the sharded FindMatches on the HIP engine.

Launched by tests/test_gpu_shard.py as
    python -m torch.distributed.run --nproc-per-node R ... tests/gpu_shard_find_worker.py OUTDIR G n p w T [flags]
Every rank runs its genome block (or, with flag "slices", its genome position slice) on cuda:0
(one GPU on the test box; exchanges over gloo) and saves its part of the MatchList (its
hash-bucket range, bucket-major).  Flag "abi": the whole pipeline runs inside the C ABI
(mums_shard_run, shard_comm.hip) with the gloo group as its transport (mums_comm_init_host);
flag "gapped": N-gapped genomes (MER_REPEAT_LIMIT restarts across the ranks); flag "compatC":
ParallelMemHash with CHUNK_SIZE C (with "abi").
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from libmems_amd.shard import HipShardEngine, ShardedFindMatches, genome_blocks, genome_slices  # noqa: E402
from libmems_amd.shard import AbiShardStage  # noqa: E402
from oracle import oracle  # noqa: E402
from tests import repeat_inputs  # noqa: E402


def genomes(G, n, p, flags):
    if "gapped" in flags:
        return repeat_inputs.n_gapped(G=G, n=n, gaps=((n // 5, 3000), (n // 2, 2500)), p=p, shift=400, seed=9)
    return oracle.generate(G, n, p, 4242 + G)


def main():
    outdir, G, n, p, w, T = (sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4]), int(sys.argv[5]),
                             int(sys.argv[6]))
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    flags = sys.argv[7:]
    seqs = genomes(G, n, p, flags)
    seed = oracle.get_seed(w)
    dev = torch.device("cuda", 0)
    lens = [len(s) for s in seqs]
    if "slices" in flags:
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
    compat = [int(f[6:]) for f in flags if f.startswith("compat")]
    if compat:   # ParallelMemHash over the ranks (chunk-range searches)
        eng.mh._check(eng.mh._lib.mums_set_parallel_compat(eng.mh._ctx, 1, compat[0]))
    if "abi" in flags:
        stage = AbiShardStage(eng, 0, stage=2, comm="host")
        stage.run_find()
        ml = eng.mh.GetMatchList()
        stage.close()
    else:
        ml = ShardedFindMatches(eng).run()
    st = eng.stats()
    np.save(os.path.join(outdir, f"len{rank}.npy"), ml.lengths)
    np.save(os.path.join(outdir, f"st{rank}.npy"), ml.starts)
    np.save(os.path.join(outdir, f"stats{rank}.npy"), np.array([st["mem_count"], st["collision_count"]]))
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
