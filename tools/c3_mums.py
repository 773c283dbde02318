"""Development driver: full FindMatches on BASELINE config 3 (8 x 100 Mbp related, w19),
generated on the GPU as bench.py does; prints the phase split.  Run under rocprofv3 to get
the per-kernel trace of the MUMs/s path:  python tools/c3_mums.py [iters] [G] [n_mbp]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import libmems_amd as lm  # noqa: E402
from bench import synth_genomes  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
n = int(float(sys.argv[3]) * 1e6) if len(sys.argv) > 3 else 100_000_000
dev = torch.device("cuda", 0)
seqs = synth_genomes(G, n, 0.01, 12345, dev)
with lm.MemHash(0) as mh:
    mh.SetSeed(lm.getSeed(19))
    for s in seqs:
        mh.AddSequence(s)
    for i in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mh.CreateMatches()
        torch.cuda.synchronize()
        st = mh.stats()
        print(f"iter {i}: {1e3 * (time.perf_counter() - t0):.1f} ms, {st['mem_count']} matches, "
              f"{st['probes']} probes, {st['chains']} chains; "
              + " ".join(f"{k}={st[k]:.2f}" for k in ("ms_keys", "ms_sort", "ms_groups", "ms_buckets",
                                                     "ms_chains", "ms_replay", "ms_output")), flush=True)
