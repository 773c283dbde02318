"""Debug: one FindMatches vs the oracle (tests' first known-answer shape); env selects the paths."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import libmems_amd as lm
from oracle import oracle
G, n, p, w = [float(x) if i == 2 else int(x) for i, x in enumerate(sys.argv[1:5])] if len(sys.argv) > 4 else (2, 1_000_000, 0.01, 15)
seqs = oracle.generate(G, n, p, 12345)
seed = oracle.get_seed(w)
L, S, st = oracle.find_matches(seqs, seed)
with lm.MemHash(0) as mh:
    mh.SetSeed(seed)
    ml = mh.FindMatches(seqs)
ok = len(ml) == len(L) and (ml.lengths == L).all() and (ml.starts == S).all()
print(os.environ.get("MUMS_DEV_KEY_ROWS"), os.environ.get("MUMS_DEV_LINE_RADIX"), "ok" if ok else "DIFF", len(ml), len(L))
if not ok and len(ml) == len(L):
    d = np.nonzero((ml.lengths != L) | (ml.starts != S).any(1))[0]
    print(len(d), "rows differ; first:", [(int(ml.lengths[i]), ml.starts[i].tolist(), int(L[i]), S[i].tolist()) for i in d[:5]])
