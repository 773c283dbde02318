"""Development probe: ParallelMemHash compat FindMatches on G related genomes of growing
length (bench.synth_genomes, w19), one line per size with the phase split:
    python tools/dev/compat_scale.py G mbp [mbp ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import libmems_amd as lm  # noqa: E402
from bench import synth_genomes  # noqa: E402

G = int(sys.argv[1])
dev = torch.device("cuda", 0)
for mbp in sys.argv[2:]:
    n = int(float(mbp) * 1e6)
    seqs = synth_genomes(G, n, 0.01, 12345, dev)
    for compat in (False, True):
        cls = (lambda: lm.ParallelMemHash(0, 200_000)) if compat else (lambda: lm.MemHash(0))
        with cls() as mh:
            mh.SetSeed(lm.getSeed(19))
            for s in seqs:
                mh.AddSequence(s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mh.CreateMatches()
            torch.cuda.synchronize()
            st = mh.stats()
        print(f"{'compat' if compat else 'memhash'} {G} x {mbp} Mbp: {1e3 * (time.perf_counter() - t0):.1f} ms, "
              f"{st['mem_count']} matches, {st['probes']} probes, chunks {st.get('chunks')}, "
              + " ".join(f"{k}={st[k]:.2f}" for k in ("ms_keys", "ms_sort", "ms_groups", "ms_buckets", "ms_chains",
                                                        "ms_replay", "ms_output")), flush=True)
    del seqs
