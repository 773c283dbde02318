"""Seed-stage time per seed pattern at BASELINE config 3 (8 x 100 Mbp related, 1 GPU).

The default-weight seeds (getSeed(15), getSeed(19)) have compiled-in run tables; the
others take the run table from the kernel argument.  This prints one JSON line per
pattern: ms per FindStage(STAGE_SEEDS) (best of K after a warm run) and the phase split,
so the two code paths can be compared inside one gpurun call.

    python tools/seed_patterns_bench.py [--steps K] [--length N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import libmems_amd as lm  # noqa: E402
from bench import synth_genomes  # noqa: E402

# (weight, rank): getSeed(19) is the bench's; ranks 1-2 are ProgressiveAligner's
# seed families (ProgressiveAligner.cpp:619-625); w11-w17 the default weights of
# smaller genomes; w21 (genomes above ~1.07 Gbp) the 8-bit scatter + msd_split.
PATTERNS = [(19, 0), (19, 1), (19, 2), (18, 0), (17, 0), (16, 0), (15, 0), (15, 1), (13, 0), (11, 0), (21, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--genomes", type=int, default=8)
    ap.add_argument("--length", type=int, default=100_000_000)
    ap.add_argument("--lib", default=None, help="A/B: another build of libmums_hip.so")
    ap.add_argument("--tag", default="")
    ap.add_argument("--patterns", default="", help="subset, e.g. 21:0,19:0")
    args = ap.parse_args()
    pats = [tuple(int(x) for x in p.split(":")) for p in args.patterns.split(",")] if args.patterns else PATTERNS
    if args.lib:
        lm.load_library(os.path.join(ROOT, args.lib))
    dev = torch.device("cuda", 0)
    genomes = synth_genomes(args.genomes, args.length, 0.01, 12345, dev)
    for w, r in pats:
        pat = lm.getSeed(w, r)
        with lm.MemHash(0) as mh:
            mh.SetSeed(pat)
            for s in genomes:
                mh.AddSequence(s)
            mh.FindStage(lm.STAGE_SEEDS)   # warm
            best = float("inf")
            for _ in range(args.steps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                mh.FindStage(lm.STAGE_SEEDS)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            mh.SetProfiling(True)
            mh.FindStage(lm.STAGE_SEEDS)
            st = mh.stats()
            mh.SetProfiling(False)
        print(json.dumps({"tag": args.tag, "weight": w, "rank": r, "pattern": hex(pat), "ms": round(best * 1e3, 3),
                          "seedmers_per_s": st["seedmers"] / best,
                          "phase_ms": {k: round(st[k], 3) for k in ("ms_keys", "ms_sort", "ms_groups", "ms_buckets")}}),
              flush=True)


if __name__ == "__main__":
    main()
