"""Development driver: the sharded FindMatches exchange at BASELINE config 3 (8 x 100 Mbp
related, w19) over W in-process ranks on one GPU (ShardedMemHash, host-staged communicator),
kept-probe export (default) against every row (MUMS_DEV_SHARD_ALL_ROWS=1): per rank the probes
it labelled, the AddHashEntry calls of its buckets, the rows / bytes it received and sent, and
the MatchList against the single-GPU one (md5 of both).
    python tools/dev/shard_exchange_c3.py W [n]"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import libmems_amd as lm  # noqa: E402
from bench import synth_genomes  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
seqs = [s.cpu().numpy().tobytes() for s in synth_genomes(8, n, 0.01, 12345, torch.device("cuda", 0))]
seed = lm.getSeed(19)


def digest(ml):
    h = hashlib.md5()
    h.update(ml.lengths.tobytes())
    h.update(ml.starts.tobytes())
    return h.hexdigest()


with lm.MemHash(0) as mh:
    mh.SetSeed(seed)
    ml1 = mh.FindMatches(seqs)
    st1 = mh.stats()
    d1 = digest(ml1)
    print(f"single GPU: {len(ml1)} matches, {st1['probes']} probes, {st1['collision_count']} collisions", flush=True)
for mode in ("kept", "all"):
    if mode == "all":
        os.environ["MUMS_DEV_SHARD_ALL_ROWS"] = "1"
    with lm.ShardedMemHash([0] * W, comm="local") as sh:
        sh.SetSeed(seed)
        t0 = time.perf_counter()
        mlw = sh.FindMatches(seqs)
        t1 = time.perf_counter()
        coll = sum(s["collision_count"] for s in sh.stats_per_rank)
        print(f"{W} ranks, {mode} rows: {len(mlw)} matches, equal {digest(mlw) == d1}, collisions {coll} "
              f"(single {st1['collision_count']}), {1e3 * (t1 - t0):.0f} ms (in-process ranks on one GPU)", flush=True)
        for r in range(W):
            ci, x, s = sh.chain_info[r], sh.exchange_info[r], sh.stats_per_rank[r]
            print(f"  rank {r}: labelled {ci['probes']}, owned calls {s['probes']}, replayed rows {ci['owned_rows']}, "
                  f"recv {x['recv_rows']} rows / {x['recv_bytes'] / 1e6:.1f} MB, sent {x['sent_rows']} rows / "
                  f"{x['sent_bytes'] / 1e6:.1f} MB", flush=True)
