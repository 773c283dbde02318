"""Development driver: ParallelMemHash compat FindMatches on BASELINE config 3 (8 x 100 Mbp
related, w19), one context, `iters` calls (the first warms the buffers); phase split per
call.  Run under rocprofv3 for the compat kernel trace:  python tools/dev/compat_c3.py [iters]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import libmems_amd as lm  # noqa: E402
from bench import synth_genomes  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
seqs = synth_genomes(8, 100_000_000, 0.01, 12345, torch.device("cuda", 0))
with lm.ParallelMemHash(0, 200_000) as mh:
    mh.SetSeed(lm.getSeed(19))
    for s in seqs:
        mh.AddSequence(s)
    for i in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        mh.CreateMatches()
        torch.cuda.synchronize()
        st = mh.stats()
        print(f"iter {i}: {1e3 * (time.perf_counter() - t0):.1f} ms, {st['mem_count']} matches, chunks {st['chunks']} "
              + " ".join(f"{k}={st[k]:.2f}" for k in ("ms_keys", "ms_sort", "ms_groups", "ms_buckets", "ms_chains",
                                                        "ms_replay", "ms_output")), flush=True)
