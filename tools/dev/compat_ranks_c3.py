"""Development driver: ParallelMemHash compat over W in-process ranks on one GPU
(ShardedMemHash(parallel_compat=True), host-staged communicator) at BASELINE config 3
(8 x 100 Mbp related, w19) against the single-GPU compat MatchList (md5 of both).
MUMS_DEV_COMPAT_RANK_DEBUG=1 prints the owners' merge steps.
    python tools/dev/compat_ranks_c3.py W [n]"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import libmems_amd as lm  # noqa: E402
from bench import synth_genomes  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
seqs = [s.cpu().numpy().tobytes() for s in synth_genomes(8, n, 0.01, 12345, torch.device("cuda", 0))]
seed = lm.getSeed(19)


def digest(ml):
    h = hashlib.md5()
    h.update(ml.lengths.tobytes())
    h.update(ml.starts.tobytes())
    return h.hexdigest()


with lm.ParallelMemHash(0, 200_000) as mh:
    mh.SetSeed(seed)
    t0 = time.perf_counter()
    ml1 = mh.FindMatches(seqs)
    t1 = time.perf_counter()
    print(f"single GPU: {len(ml1)} matches, {1e3 * (t1 - t0):.0f} ms (first call), chunks {mh.stats()['chunks']}",
          flush=True)
    d1 = digest(ml1)
for it in range(2):
    with lm.ShardedMemHash([0] * W, comm="local", parallel_compat=True, chunk_size=200_000) as sh:
        sh.SetSeed(seed)
        t0 = time.perf_counter()
        mlw = sh.FindMatches(seqs)
        t1 = time.perf_counter()
        per = [(s["probes"], s["mem_count"]) for s in sh.stats_per_rank]
        print(f"{W} ranks (call {it}): {len(mlw)} matches, {1e3 * (t1 - t0):.0f} ms, equal {digest(mlw) == d1}, "
              f"(probes, entries) per rank {per}", flush=True)
