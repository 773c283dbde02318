#!/usr/bin/env python3
"""BASELINE config 5 on one MI355X: 2 x 3 Gbp related synthetic genomes, seed weight 19,
MemHash seed stage ("sorted+matched") in the chunked mode (> 2^32 seed-mers per context,
libmems_amd/csrc/chunked.hip).  Reports seed-mers/s and, as size-independent parity
checks, that a finer chunking (MUMS_DEV_CHUNK_RECORDS) gives the same probe and group
counts, and that the run is repeatable.  Then the whole FindMatches (2.5e9 AddHashEntry
calls: chains per 2^28-probe slice, replay in chunks of the bucket order) timed likewise.

    python tools/bench_c5.py [--length 3000000000] [--steps 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import libmems_amd as lm  # noqa: E402


def synth_pair(n: int, p: float, seed: int, dev):
    """genome 0 iid ACGT; genome 1 = genome 0 with substitution rate p (chunked generation)."""
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    a = torch.empty(n, dtype=torch.uint8, device=dev)
    b = torch.empty(n, dtype=torch.uint8, device=dev)
    step = 1 << 28
    for o in range(0, n, step):
        k = min(step, n - o)
        x = lut[torch.randint(0, 4, (k,), generator=gen, device=dev, dtype=torch.uint8).long()]
        a[o:o + k] = x
        mut = torch.rand(k, generator=gen, device=dev) < p
        sub = lut[torch.randint(0, 4, (k,), generator=gen, device=dev, dtype=torch.uint8).long()]
        b[o:o + k] = torch.where(mut, sub, x)
    torch.cuda.synchronize()
    return a, b


def add_gaps(a, b, gaps: int, seed: int):
    """N runs as in assembled mammalian genomes: `gaps` runs of 5-60 kbp per genome at random
    positions (N encodes as A: each run is one seed group of tens of thousands of records,
    a MER_REPEAT_LIMIT restart, MatchFinder.cpp:253-277)."""
    g = torch.Generator()
    g.manual_seed(seed)
    n = a.numel()
    for t in (a, b):
        pos = torch.randint(0, n - 60_000, (gaps,), generator=g).tolist()
        ln = torch.randint(5_000, 60_000, (gaps,), generator=g).tolist()
        for p0, l0 in zip(pos, ln):
            t[p0:p0 + l0] = ord("N")
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--length", type=int, default=3_000_000_000)
    ap.add_argument("--weight", type=int, default=19, help="seed weight (21 = getDefaultSeedWeight of 3 Gbp genomes)")
    ap.add_argument("--gaps", type=int, default=0, help="N runs per genome (restarts)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--fine-cap", type=int, default=400_000_000)
    ap.add_argument("--find-steps", type=int, default=2)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    a, b = synth_pair(args.length, 0.01, 2024, dev)
    if args.gaps:
        add_gaps(a, b, args.gaps, 77)
    gen_s = time.perf_counter() - t0
    print(f"generated 2 x {args.length} bp in {gen_s:.1f} s", flush=True)
    out = {"config": "BASELINE config 5 shape on 1 GPU: 2 x %d bp related p=0.01, w%d (%s)%s, MemHash seed stage"
                     % (args.length, args.weight, hex(lm.getSeed(args.weight)),
                        f", {args.gaps} N runs of 5-60 kbp per genome" if args.gaps else "")}
    with lm.MemHash(0) as mh:
        mh.SetSeed(lm.getSeed(args.weight))
        mh.AddSequence(a)
        mh.AddSequence(b)
        mh.FindStage(lm.STAGE_SEEDS)   # warm
        print("warm run done", flush=True)
        ts = []
        for _ in range(args.steps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            mh.FindStage(lm.STAGE_SEEDS)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t1)
            print(f"step {ts[-1] * 1e3:.1f} ms", flush=True)
        st = mh.stats()
        os.environ["MUMS_DEV_CHUNK_RECORDS"] = str(args.fine_cap)
        mh.FindStage(lm.STAGE_SEEDS)
        fine = mh.stats()
        os.environ.pop("MUMS_DEV_CHUNK_RECORDS")
        fts = []
        for _ in range(args.find_steps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            mh.CreateMatches()
            torch.cuda.synchronize()
            fts.append(time.perf_counter() - t1)
            print(f"FindMatches {fts[-1] * 1e3:.1f} ms", flush=True)
        fst = mh.stats() if fts else None
    dt = min(ts)
    out.update({
        "seedmers": st["seedmers"], "seedmers_per_s": st["seedmers"] / dt, "ms_per_step": dt * 1e3,
        "chunks": st["chunks"], "probes": st["probes"], "groups": st["groups"],
        "phase_ms": {k: round(st[k], 2) for k in ("ms_keys", "ms_sort", "ms_groups", "ms_buckets", "ms_total")},
        "finer_chunking": {"chunks": fine["chunks"], "probes": fine["probes"], "groups": fine["groups"],
                           "same_counts": (fine["probes"], fine["groups"]) == (st["probes"], st["groups"])},
    })
    if fst:
        fd = min(fts)
        out["findmatches"] = {
            "ms": fd * 1e3, "matches": fst["mem_count"], "mums_per_s": fst["mem_count"] / fd, "probes": fst["probes"],
            "chains": fst["chains"], "mem_count": fst["mem_count"], "collisions": fst["collision_count"],
            "restarts": fst.get("restarts"), "repeat_limit_groups": fst.get("repeat_limit_groups"),
            "phase_ms": {k: round(fst[k], 2) for k in fst if k.startswith("ms_")},
        }
    print(json.dumps(out), flush=True)
    if not out["finer_chunking"]["same_counts"]:
        sys.exit(3)


if __name__ == "__main__":
    main()
