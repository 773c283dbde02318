"""Development measurement: the sharded MER_REPEAT_LIMIT restart planned on every rank's own
SortedMerList parts (default) vs gathered onto rank 0 (MUMS_DEV_SHARD_RESTART=gather), on
N-gapped related genomes over W in-process ranks of one GPU (host-staged communicator, so
the exchange times are not xGMI's).  Per path: FindMatches wall time, matches, restarts and
every rank's restart buffers (mums_shard_restart_info)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libmems_amd as lm  # noqa: E402
from oracle import oracle  # noqa: E402
from tests import repeat_inputs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--genomes", type=int, default=2)
ap.add_argument("--length", type=int, default=20_000_000)
ap.add_argument("--gaps", type=int, default=40)
ap.add_argument("--world", type=int, default=4)
ap.add_argument("--weight", type=int, default=19)
ap.add_argument("--layout", default="slices")
ap.add_argument("--modes", default="local,gather,local")
a = ap.parse_args()
import threading  # noqa: E402


def heartbeat():   # (gpurun takes 3 silent minutes for a hang)
    t0 = time.time()
    while True:
        time.sleep(30)
        print(f"... {time.time() - t0:.0f} s", flush=True)


threading.Thread(target=heartbeat, daemon=True).start()
n = a.length
gaps = tuple((int((i + 0.5) * n / a.gaps), 5000) for i in range(a.gaps))
seqs = repeat_inputs.n_gapped(G=a.genomes, n=n, gaps=gaps, shift=700, seed=5)
print("inputs ready", flush=True)
out = {"genomes": a.genomes, "length": n, "gaps": a.gaps, "world": a.world, "weight": a.weight, "layout": a.layout}
for mode in a.modes.split(","):
    if mode == "gather":
        os.environ["MUMS_DEV_SHARD_RESTART"] = "gather"
    else:
        os.environ.pop("MUMS_DEV_SHARD_RESTART", None)
    with lm.ShardedMemHash([0] * a.world, comm="local", layout=a.layout) as sh:
        sh.SetSeed(oracle.get_seed(a.weight))
        t0 = time.perf_counter()
        ml = sh.FindMatches(seqs)
        dt = time.perf_counter() - t0
        info = sh.restart_info
        out[mode] = {"s": round(dt, 3), "seedmers": sum(st["seedmers"] for st in sh.stats_per_rank), "matches": len(ml), "restarts": sh.stats_per_rank[0]["restarts"],
                     "restart_bytes_per_rank": [i["bytes"] for i in info], "path": [i["path"] for i in info],
                     "candidates": [i["candidates"] for i in info]}
    print(mode, json.dumps(out[mode]), flush=True)
print(json.dumps(out))
