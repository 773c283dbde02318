"""Development: GPU FindMatches on the C3 known-answer input (tests/golden/large_cases.json),
timed, with the stats the test compares.   python tools/c3_golden_check.py [case]"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import libmems_amd as lm  # noqa: E402
from oracle import oracle  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
c = json.load(open(os.path.join(ROOT, "tests", "golden", "large_cases.json")))[name]
t0 = time.time()
seqs = oracle.generate(c["G"], c["n"], c["p"], c["gen_seed"])
print(f"generated in {time.time() - t0:.1f} s", flush=True)
dev = [torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda() for s in seqs]
del seqs
torch.cuda.synchronize()
with lm.MemHash(0) as mh:
    mh.SetSeed(c["seed"])
    for s in dev:
        mh.AddSequence(s)
    for it in range(2):
        t1 = time.time()
        mh.CreateMatches()
        torch.cuda.synchronize()
        st = mh.stats()
        print(f"FindMatches {1e3 * (time.time() - t1):.1f} ms", {k: st[k] for k in ("seedmers", "probes", "mem_count",
              "collision_count", "restarts", "chains", "ms_chains", "ms_replay")}, flush=True)
    ml = mh.GetMatchList()
md5 = hashlib.md5(ml.text().encode()).hexdigest()
print("md5", md5, "expected", c["md5"], "matches", len(ml), "expected", c["matches"], "OK" if md5 == c["md5"] else "DIFF")
