"""Development check of the sharded chain labelling (mums_shard_chain_*) against the
oracle and the bucket-owner layout on one small input; prints per-rank counts."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import libmems_amd as lm  # noqa: E402
from oracle import oracle  # noqa: E402

G, n, w, p = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
seqs = oracle.generate(G, n, p, 12345)
seed = oracle.get_seed(w)
L, S, st = oracle.find_matches(seqs, seed)
print("oracle", len(L), st["collision_count"])
for world in (1, 2):
    for mode in ("labelled", "bucket"):
        if mode == "bucket":
            os.environ["MUMS_DEV_SHARD_BUCKET_CHAINS"] = "1"
        else:
            os.environ.pop("MUMS_DEV_SHARD_BUCKET_CHAINS", None)
        with lm.ShardedMemHash([0] * world, comm="local") as sh:
            sh.SetSeed(seed)
            ml = sh.FindMatches(seqs)
            eq = len(ml) == len(L) and np.array_equal(ml.lengths, L) and np.array_equal(ml.starts, S)
            print(world, mode, len(ml), eq, [(s["probes"], s["chains"], s["collision_count"]) for s in sh.stats_per_rank],
                  getattr(sh, "chain_info", None))
with lm.MemHash(0) as mh:
    mh.SetSeed(seed)
    for mode in ("one", "sliced"):
        if mode == "sliced":
            os.environ["MUMS_DEV_FIND_CHUNK"] = "5000"
        ml = mh.FindMatches(seqs)
        s = mh.stats()
        print("single", mode, len(ml), len(ml) == len(L) and np.array_equal(ml.lengths, L), s["probes"], s["chains"])
