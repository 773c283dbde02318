"""Development diagnostic: sharded seed stage (gloo, all ranks on cuda:0) vs single GPU
on synthetic related genomes generated on the GPU (bench.py's generator)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import torch.distributed as dist
import libmems_amd as lm
from libmems_amd.shard import HipShardEngine, ShardedSeedStage, genome_blocks
from bench import synth_genomes

G, n = int(sys.argv[1]), int(sys.argv[2])
out = sys.argv[3]
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
seed = lm.getSeed(19)
g = synth_genomes(G, n, 0.01, 12345, dev)
first, count = genome_blocks(G, world)[rank]
eng = HipShardEngine(0, seed, [n] * G, first, g[first:first + count])
st_ = ShardedSeedStage(eng)
st_.run()
b, r = eng.probes()
s = eng.stats()
print(f"rank {rank}: range {st_.last_range} recs {s['seedmers']} groups {s['groups']} probes {s['probes']}", flush=True)
np.save(f"{out}/b{rank}.npy", b); np.save(f"{out}/r{rank}.npy", r)
dist.barrier()
if rank == 0:
    with lm.MemHash(0) as mh:
        mh.SetSeed(seed)
        for x in g:
            mh.AddSequence(x)
        mh.FindStage(lm.STAGE_SEEDS)
        sb, sr = mh.Probes()
        ss = mh.stats()
    bb = np.concatenate([np.load(f"{out}/b{k}.npy") for k in range(world)])
    rr = np.concatenate([np.load(f"{out}/r{k}.npy") for k in range(world)])
    print("single: groups", ss["groups"], "probes", ss["probes"], "| sharded total", len(bb),
          "equal:", len(bb) == len(sb) and bool(np.array_equal(bb, sb) and np.array_equal(rr, sr)), flush=True)
dist.destroy_process_group()
