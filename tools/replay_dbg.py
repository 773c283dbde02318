"""Development: time FindMatches on the BASELINE config-2 shape with replay instrumentation."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libmems_amd as lm
from bench import synth_genomes
dev = torch.device("cuda", 0)
G = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
p = float(sys.argv[3]) if len(sys.argv) > 3 else 0.01
seqs = synth_genomes(G, n, p, 777, dev)
with lm.MemHash(0) as mh:
    mh.SetSeed(lm.getSeed(15))
    for s in seqs:
        mh.AddSequence(s)
    for it in range(2):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        mh.CreateMatches(); torch.cuda.synchronize()
        st = mh.stats()
        print(f"iter {it}: {1e3*(time.perf_counter()-t0):.1f} ms, matches {st['mem_count']}, chains {st['chains']}, "
              f"probes {st['probes']}, ms_chains {st['ms_chains']:.2f} ms_replay {st['ms_replay']:.2f}", flush=True)
