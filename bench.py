#!/usr/bin/env python3
"""Benchmark: seed-mers/s sorted+matched on BASELINE config 3 (8 x 100 Mbp, w19) per MI355X.

One step = one pass of the MemHash seed hot path over the whole input: canonical
spaced-seed keys for every position of every genome, the radix sort that builds
the G SortedMerLists merged into one key-ordered stream, the equal-key group scan
with MemHash acceptance, probe construction (SetDirection, CalculateOffset) and the
stable bucket partition of the probes (SURVEY.md 8(d) "sorted+matched").  Inputs
(ASCII genomes) are resident in HBM before the timed region.  MUMs/s (full
FindMatches incl. extension, bucket replay and MatchList output) is reported
beside it on BASELINE config 2 (4 x 10 Mbp, w15).

    python bench.py [--gpus N --steps K --warmup W]
For N > 1 launch with torch.distributed.run (one rank per GPU): the same C3 input is
split genome-block-per-rank and the seed stage runs sharded (libmems_amd/shard.py:
keys per rank, RCCL all-to-all of key ranges, merge per key range), so the total
work is fixed ("strong" scaling) and value = all seed-mers / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (loaded before libmums_hip.so: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

import libmems_amd as lm  # noqa: E402
from libmems_amd.shard import AbiShardStage, HipShardEngine, ShardedSeedStage, genome_blocks, genome_slices  # noqa: E402

METRIC = "seed-mers/sec sorted+matched (+ MUMs/sec) at 1/2/4/8 MI355X; HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
# the newest round's PMC summary of the dominant kernel (tools/round_evidence.sh + summarize_profile.py)
_SUMMARIES = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]*_dominant_kernel.json")))
PROFILE_SUMMARY = _SUMMARIES[-1] if _SUMMARIES else os.path.join(ROOT, "profiles", "r01_dominant_kernel.json")


_T0 = time.perf_counter()


def progress(msg: str) -> None:
    """Progress line on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench +{time.perf_counter() - _T0:.1f}s] {msg}", file=sys.stderr, flush=True)


def synth_genomes(G: int, n: int, p: float, seed: int, device: torch.device):
    """Synthetic related genomes on the GPU: genome 0 iid ACGT; genome g>0 = genome 0 with
    per-base substitution rate p; genome 2 reverse-complemented (SURVEY.md 8(d) shape)."""
    if n > (1 << 28):
        return synth_genomes_large(G, n, p, seed, device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=device)
    comp = torch.zeros(256, dtype=torch.uint8, device=device)
    for a, b in zip(b"ACGT", b"TGCA"):
        comp[a] = b
    base = lut[torch.randint(0, 4, (n,), generator=gen, device=device, dtype=torch.int64)]
    out = [base]
    for g in range(1, G):
        mask = torch.rand(n, generator=gen, device=device) < p
        sub = lut[torch.randint(0, 4, (n,), generator=gen, device=device, dtype=torch.int64)]
        s = torch.where(mask, sub, base)
        if g == 2:
            s = comp[s.flip(0).long()]
        out.append(s.contiguous())
    torch.cuda.synchronize()
    return out


def synth_genomes_large(G: int, n: int, p: float, seed: int, device: torch.device):
    """synth_genomes for mammalian-scale n (BASELINE config 5), generated 2^28 bases at a
    time; no reverse complement (config 5 has two genomes)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    lut = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=device)
    out = [torch.empty(n, dtype=torch.uint8, device=device) for _ in range(G)]
    step = 1 << 28
    for o in range(0, n, step):
        k = min(step, n - o)
        x = lut[torch.randint(0, 4, (k,), generator=gen, device=device, dtype=torch.uint8).long()]
        out[0][o:o + k] = x
        for g in range(1, G):
            mut = torch.rand(k, generator=gen, device=device) < p
            sub = lut[torch.randint(0, 4, (k,), generator=gen, device=device, dtype=torch.uint8).long()]
            out[g][o:o + k] = torch.where(mut, sub, x)
    torch.cuda.synchronize()
    return out


def cpu_threads() -> int:
    """Host threads of the CPU baseline: the GPU box's CPU share (16 per GPU), capped by
    the CPUs this process may run on."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline():
    """OpenMP CPU path (oracle_find_matches_omp: per-genome SMLs in parallel, merge split by
    key range; bit-identical to the serial restatement) on the host cores, seed stage of
    BASELINE config 3 itself (8 x 100 Mbp related, w19)."""
    from oracle import oracle

    G, n, p = 8, 100_000_000, 0.01
    th = cpu_threads()
    seqs = oracle.generate(G, n, p, 12345)
    seed = lm.getSeed(19)
    t0 = time.perf_counter()
    _, _, st = oracle.seed_probes(seqs, seed, omp_threads=th)
    dt = time.perf_counter() - t0
    return {
        "value": st["seedmers"] / dt,
        "unit": "seed-mers/s",
        "cores": th,
        "kind": "port",
        "cpu": cpu_model(),
        "sample": f"OpenMP oracle MemHash seed stage (keys + per-genome SML sort in parallel, G-way merge split "
                  f"by key range, acceptance, probes + buckets), BASELINE config 3 itself: {G} x {n // 10**6} Mbp "
                  f"related p={p}, w19 seed 0x7b974ef, {st['seedmers']} seed-mers in {dt:.1f} s, {th} threads",
    }


def cpu_baseline_mums():
    """OpenMP oracle FindMatches (bucket replay in parallel, same MatchList as serial) on
    the config-2 shape itself (4 x 10 Mbp related, w15)."""
    from oracle import oracle

    G, n, p = 4, 10_000_000, 0.01
    th = cpu_threads()
    seqs = oracle.generate(G, n, p, 12345)
    t0 = time.perf_counter()
    lengths, _, _ = oracle.find_matches(seqs, lm.getSeed(15), omp_threads=th)
    dt = time.perf_counter() - t0
    return {"value": len(lengths) / dt, "unit": "MUMs/s", "cores": th, "kind": "port", "cpu": cpu_model(),
            "sample": f"OpenMP oracle MemHash::FindMatches (SMLs, merge by key range, ExtendMatch + AddHashEntry "
                      f"per hash bucket in parallel), {G} x {n // 10**6} Mbp related p={p}, w15, {len(lengths)} "
                      f"matches in {dt:.1f} s, {th} threads"}


def run_mums(device: int, dev: torch.device, p: float = 0.01, reps: int = 3):
    """MUMs/s on BASELINE config 2 (4 x 10 Mbp, w15): full FindMatches (seed stage, chain
    labelling, bucket replay, MatchList on the device); best of `reps` after a warm run."""
    seqs = synth_genomes(4, 10_000_000, p, 777, dev)
    with lm.MemHash(device) as mh:
        mh.SetSeed(lm.getSeed(15))
        for s in seqs:
            mh.AddSequence(s)
        mh.CreateMatches()  # warm
        dt = float("inf")
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mh.CreateMatches()
            torch.cuda.synchronize()
            dt = min(dt, time.perf_counter() - t0)
        st = mh.stats()
    kind = "related p=0.01" if p < 1.0 else "iid (unrelated)"
    return {"mums_per_s": st["mem_count"] / dt, "matches": st["mem_count"], "ms": dt * 1e3,
            "workload": f"4 x 10 Mbp {kind}, w15 (BASELINE config 2 shape), full FindMatches",
            "phase_ms": {k: round(st[k], 3) for k in ("ms_keys", "ms_sort", "ms_groups", "ms_buckets", "ms_chains", "ms_replay",
                                                        "ms_output")}}


_WALK_PMCS = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_chains.txt")))
WALK_PMC = _WALK_PMCS[-1] if _WALK_PMCS else os.path.join(ROOT, "profiles", "r04v_pmc_chains.txt")


def walk_counter_traffic(walk_ms, kernel="chain_walk_kernel"):
    """A walk kernel's HBM-side bytes from the committed rocprofv3 PMC passes
    (tools/pmc_chains.sh: FETCH_SIZE + WRITE_SIZE per dispatch, KiB, not this run) over the
    live duration of its two launches: the counter-based roofline next to the requested one."""
    try:
        per = {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0}
        seen = 0
        for line in open(WALK_PMC):   # "<kernel> <counter> <value per dispatch>", kernel names may hold spaces
            f = line.rsplit(None, 2)
            if len(f) == 3 and f[0].startswith(kernel + "<") and f[1] in per:
                per[f[1]] += float(f[2]) * 1024
                seen += 1
        if not seen:
            raise KeyError(kernel)
        b = 2 * (per["FETCH_SIZE"] + per["WRITE_SIZE"])   # each instance: one launch per pass, two passes
        gbs = b / (walk_ms * 1e-3) / 1e9
        return {"traffic": b, "traffic_achieved": gbs, "traffic_frac": gbs / HBM_PEAK_GBS,
                "traffic_source": os.path.relpath(WALK_PMC, ROOT) + f" (FETCH_SIZE + WRITE_SIZE per dispatch of "
                                  f"every {kernel} instance x 2 passes, rocprofv3 PMC passes, not this run)"}
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return {"traffic": None}


def walk_roofline(kernel, ms, nbytes, walks, words, what):
    """Requested-bytes roofline of one walk kernel (HIP events around its two launches) with
    the committed counter bytes beside it."""
    gbs = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else None
    return {"bound": "hbm", "kernel": kernel + " (2 launches per FindMatches, " + what + ")",
            "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS if gbs else None,
            "bytes": nbytes, "ms": ms, "walks": walks, "hit_words": words,
            "model": "REQUESTED bytes: 28-B packed window per 64-column hit word and present component + per walk "
                     "the probe row (int32 starts, 32 B at G=8) and its 24-B queue item; much of the 200 MB packed "
                     "genome is served from L2 / MALL",
            **(walk_counter_traffic(ms, kernel) if ms > 0 else {"traffic": None})}


def run_compat(device: int, genomes, seed, reps: int = 2):
    """ParallelMemHash (ParallelMemHash.cpp:42-121, CHUNK_SIZE 200 000) on the metric's config:
    the patched OpenMP reference's MatchList (chunked search, MergeTable), full FindMatches
    from the resident genomes; best of `reps` after a warm run."""
    with lm.ParallelMemHash(device, 200_000) as mh:
        mh.SetSeed(seed)
        for s in genomes:
            mh.AddSequence(s)
        mh.CreateMatches()   # warm
        dt = float("inf")
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mh.CreateMatches()
            torch.cuda.synchronize()
            dt = min(dt, time.perf_counter() - t0)
        st = mh.stats()
    return {"mums_per_s": st["mem_count"] / dt, "matches": st["mem_count"], "ms": dt * 1e3,
            "chunks": st["chunks"], "probes": st["probes"], "restarts": st["restarts"],
            "workload": f"BASELINE config 3 ({len(genomes)} x {genomes[0].numel() // 10**6} Mbp related, w19) under "
                        f"ParallelMemHash compat (chunks of 200 000 mers of the longest SML, MergeTable), full "
                        f"FindMatches",
            "phase_ms": {k: round(st[k], 3) for k in ("ms_keys", "ms_sort", "ms_groups", "ms_buckets", "ms_chains",
                                                        "ms_replay", "ms_output")}}


def run_e2e(mh, genomes, seed, reps: int = 2):
    """End to end on the metric's config: host ASCII in pinned memory ->
    AddSequence (H2D copy into the context) -> FindMatches -> host MatchList (lengths +
    signed starts, mums_result_copy).  The context is warm (its work buffers sized by the
    runs before), as for a caller that reuses a MemHash; best of `reps`."""
    pinned = [g.cpu().pin_memory() for g in genomes]
    # the host MatchList lands in caller-owned pinned buffers (like the input), sized by the
    # warm-up run and reused by the timed ones
    out = None
    best = None
    for _ in range(reps + 1):   # the first run warms the per-genome allocations
        mh.Clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for p in pinned:
            mh.AddSequence(p)
        t1 = time.perf_counter()
        mh.SetSeed(seed)
        mh.CreateMatches()
        t2 = time.perf_counter()
        ml = mh.GetMatchList(out)
        t3 = time.perf_counter()
        r = (t3 - t0, t1 - t0, t2 - t1, t3 - t2, len(ml))
        if out is None:   # warm-up run: allocate the pinned result buffers
            n, G = len(ml), len(genomes)
            out = (torch.empty(n, dtype=torch.int64, pin_memory=True).numpy().view(np.uint64),
                   torch.empty(n * G, dtype=torch.int64, pin_memory=True).numpy())
            continue
        if best is None or r[0] < best[0]:
            best = r
    tot, add, find, copy, m = best
    sm = mh.stats()
    return {"mums_per_s": m / tot, "seedmers_per_s": sm["seedmers"] / tot, "matches": m, "ms": tot * 1e3,
            "ms_add_h2d": add * 1e3, "ms_find": find * 1e3, "ms_result_d2h": copy * 1e3,
            "workload": f"BASELINE config 3 end to end: {len(genomes)} x {genomes[0].numel() // 10**6} Mbp ASCII in "
                        f"pinned host memory -> host MatchList ({m} matches x {len(genomes)} starts) in caller-owned "
                        f"pinned buffers"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--genomes", type=int, default=8)
    ap.add_argument("--length", type=int, default=100_000_000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-mums", action="store_true")
    ap.add_argument("--no-compat", action="store_true",
                    help="skip the ParallelMemHash compat FindMatches at C3 (mums_c3_compat)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL, default) or gloo (rehearsal)")
    ap.add_argument("--exchange", choices=("abi", "torch"), default="abi",
                    help="abi (default): the C ABI runs the sharded step with its own RCCL communicator "
                         "(mums_shard_run; torch.distributed = gloo control plane); torch: records move by "
                         "torch.distributed all_to_all (shard.py)")
    ap.add_argument("--force-shard", action="store_true", help="run the sharded path even on one GPU")
    ap.add_argument("--device", type=int, default=None, help="force one HIP device for every rank (rehearsal)")
    ap.add_argument("--workload", choices=("c3", "c5"), default="c3",
                    help="c3 (default, the metric's config): 8 x 100 Mbp; c5: 2 x 3 Gbp (chunked mode on 1 GPU, "
                         "position-sharded genomes on N GPUs, N a multiple of 8)")
    args = ap.parse_args()
    if args.workload == "c5":
        args.genomes = 2
        if args.length == 100_000_000:   # not overridden: the config's 3 Gbp
            args.length = 3_000_000_000
        args.no_mums = True
        args.no_cpu_baseline = True

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) if args.device is None else args.device
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    sharded = world > 1 or args.force_shard
    if args.exchange == "abi":   # the data moves by the library's RCCL communicator
        args.dist_backend = "gloo"
    if world > 1:
        # RCCL ("nccl" on ROCm) over xGMI: the key-range all-to-all of the sharded seed stage
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    G, n = args.genomes, args.length
    seed = lm.getSeed(19)
    genomes = synth_genomes(G, n, 0.01, 12345, dev)
    phase = {"ms_keys": 0.0, "ms_sort": 0.0, "ms_groups": 0.0, "ms_buckets": 0.0}
    ms_dom = 0.0
    bytes_dom = 0
    launches = 0
    exch_bytes = 0
    abi_err = None
    if not sharded:
        mh = lm.MemHash(local)
        mh.SetSeed(seed)
        for s in genomes:
            mh.AddSequence(s)
        run = lambda: mh.FindStage(lm.STAGE_SEEDS)  # noqa: E731
        stats = mh.stats
    elif args.workload == "c5":
        # genome position slices (each 3 Gbp genome over world/G ranks)
        L = lm.getSeedLength(seed)
        g, b0, b1 = genome_slices([n] * G, L, world)[rank]
        mine = [genomes[g][b0:min(n, b1 + L - 1)]]
        eng = HipShardEngine(local, seed, [n] * G, g, mine, slice_of=(g, b0, b1))
        genomes = mine   # views into genome g keep its storage alive
        stage = AbiShardStage(eng, local) if args.exchange == "abi" else ShardedSeedStage(eng)
        mh = eng.mh
        run = stage.run
        stats = eng.stats
    else:
        # genome block per rank; the whole C3 input is split, not replicated
        first, count = genome_blocks(G, world)[rank]
        mine = genomes[first:first + count]
        del genomes
        genomes = mine
        eng = HipShardEngine(local, seed, [n] * G, first, genomes)
        if args.exchange == "abi":
            try:
                stage = AbiShardStage(eng, local)
            except Exception as e:  # agreed on below: every rank falls back together
                stage, abi_err = None, e
        else:
            stage = ShardedSeedStage(eng)
        mh = eng.mh
        run = stage.run if stage is not None else None
        stats = eng.stats
    fallback = None
    if sharded and world > 1 and args.exchange == "abi":
        # the library's own RCCL communicator has only run with one rank on the one-GPU test
        # boxes: if its first step fails on any rank, every rank (agreed over the gloo control
        # group) continues with the torch.distributed RCCL exchange of shard.py instead, and
        # the line says so
        ok = 1
        try:
            if stage is None:
                raise RuntimeError(f"communicator: {abi_err}")
            stage.run()
        except Exception as e:  # report, never hide
            ok = 0
            fallback = f"mums_shard_run failed on rank {rank}: {e}"
            print(fallback, file=sys.stderr, flush=True)
        flag = torch.tensor([ok], dtype=torch.int64)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 0:
            if fallback is None:
                fallback = "mums_shard_run failed on another rank"
            nccl = dist.new_group(backend="nccl")
            if stage is not None:
                stage.close()
            stage = ShardedSeedStage(eng, group=nccl)
            run = stage.run
            args.exchange = "torch"
            args.dist_backend = "nccl"
    for _ in range(args.warmup):
        run()

    def barrier():
        if world > 1:
            if args.dist_backend == "nccl" and fallback is None:
                dist.barrier(device_ids=[local])
            else:
                dist.barrier()

    progress(f"timed region: {args.steps} steps")
    # timed region: K steps, no per-pass instrumentation events
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
        if world > 1:
            exch_bytes += stage.last_exchange_bytes
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    tmax = torch.tensor([dt], dtype=torch.float64, device=dev if (args.dist_backend == "nccl" and fallback is None)
                        else "cpu")
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dt = float(tmax.item())
    # after it, the same K steps with HIP events around every sort-pass launch (on the
    # context's stream) for the dominant kernel's live duration and the phase split
    progress(f"timed region done: {dt / args.steps * 1e3:.3f} ms/step; profiled steps")
    mh.SetProfiling(True)
    for _ in range(args.steps):
        run()
        st = stats()
        ms_dom += st["ms_dominant"]
        bytes_dom += st["dominant_bytes"]
        launches += st["dominant_launches"]
        for k in phase:
            phase[k] += st[k]
    mh.SetProfiling(False)
    mums_c3 = None
    e2e_c3 = None
    compat_c3 = None
    if world == 1 and args.workload == "c3" and not args.no_mums:
        # MUMs/s on the metric's own config: full FindMatches of the resident C3 genomes
        progress("C3 FindMatches")
        try:
            mh.CreateMatches()   # warm
            best = float("inf")
            for _ in range(2):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                mh.CreateMatches()
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t1)
            sm = mh.stats()
            # one more FindMatches with HIP events around the dominant kernel's launches
            # (chain_walk_kernel) for its live duration and the roofline of the MUMs/s path
            mh.SetProfiling(True)
            mh.CreateMatches()
            sp = mh.stats()
            mh.SetProfiling(False)
            mums_c3 = {"mums_per_s": sm["mem_count"] / best, "matches": sm["mem_count"], "ms": best * 1e3,
                       "probes": sm["probes"], "chains": sm["chains"], "collisions": sm["collision_count"],
                       "workload": f"BASELINE config 3: {G} x {n // 10**6} Mbp related p=0.01, w19, full FindMatches",
                       "phase_ms": {k: round(sm[k], 3) for k in ("ms_keys", "ms_sort", "ms_groups", "ms_buckets",
                                                                  "ms_chains", "ms_replay", "ms_output")},
                       # FindMatches' largest kernel, then the lane-group walks it hands on to
                       "roofline": walk_roofline("chain_walk_short_kernel", sp["ms_short_walks"],
                                                 sp["short_walk_bytes"], sp["short_walks"], sp["short_walk_words"],
                                                 "every queued walk, one lane each, up to 8 words"),
                       "roofline_long_walks": walk_roofline("chain_walk_kernel", sp["ms_chain_walks"],
                                                            sp["chain_walk_bytes"], sp["chain_walks"],
                                                            sp["chain_walk_words"],
                                                            "the walks past 8 words, 16 then 64 lanes each")}
        except Exception as e:  # report, never hide
            mums_c3 = {"error": str(e)}
        progress("C3 end to end")
        try:
            e2e_c3 = run_e2e(mh, genomes, seed)
        except Exception as e:  # report, never hide
            e2e_c3 = {"error": str(e)}
        if not args.no_compat:
            progress("C3 ParallelMemHash compat")
            try:
                compat_c3 = run_compat(local, genomes, seed)
            except Exception as e:  # report, never hide
                compat_c3 = {"error": str(e)}
    elif sharded and args.workload == "c3" and not args.no_mums and hasattr(stage, "run_find"):
        # MUMs/s of the sharded FindMatches (mums_shard_run, all 8 steps: keys, record
        # all-to-allv, merge, bucket ranges, row all-to-allv, packed all-gather, chains + replay)
        # on the same split C3 input: total matches over the ranks / max-over-ranks time
        try:
            stage.run_find()   # warm
            best = float("inf")
            for _ in range(2):
                barrier()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                stage.run_find()
                torch.cuda.synchronize()
                barrier()
                best = min(best, time.perf_counter() - t1)
            sm = stats()
            red = torch.tensor([best, float(sm["mem_count"]), float(sm["probes"]), float(sm["collision_count"])],
                               dtype=torch.float64)
            tmx = red[:1].clone()
            if world > 1:
                dist.all_reduce(tmx, op=dist.ReduceOp.MAX)
                dist.all_reduce(red, op=dist.ReduceOp.SUM)
            best = float(tmx.item())
            matches = int(red[1].item())
            # every rank's chain stage: the probes it labelled (its key range) and the time
            ci = stage.chain_info() if hasattr(stage, "chain_info") else {"probes": 0, "ms": 0.0}
            per = torch.tensor([[float(ci["probes"]), ci["ms"], float(sm["probes"]), float(sm["ms_replay"]),
                                 float(ci.get("recv_rows", 0)), float(ci.get("recv_bytes", 0)),
                                 float(ci.get("sent_rows", 0)), float(ci.get("sent_bytes", 0))]], dtype=torch.float64)
            allr = [torch.zeros_like(per) for _ in range(world)] if world > 1 else [per]
            if world > 1:
                dist.all_gather(allr, per)
            # per rank: the probes it labelled, the AddHashEntry calls of its buckets (kept rows
            # received + the collisions the sources counted instead of sending), what it received
            # and sent in the FindMatches exchange (mums_comm_exchange_info)
            ranks_chain = [{"labelled_probes": int(a[0, 0].item()), "ms_label": round(float(a[0, 1].item()), 3),
                            "owned_calls": int(a[0, 2].item()), "ms_replay": round(float(a[0, 3].item()), 3),
                            "recv_rows": int(a[0, 4].item()), "recv_bytes": int(a[0, 5].item()),
                            "sent_rows": int(a[0, 6].item()), "sent_bytes": int(a[0, 7].item())}
                           for a in allr]
            mums_c3 = {"mums_per_s": matches / best, "matches": matches, "ms": best * 1e3,
                       "probes": int(red[2].item()), "collisions": int(red[3].item()),
                       "workload": f"BASELINE config 3: {G} x {n // 10**6} Mbp related p=0.01, w19, full FindMatches "
                                   f"sharded over {world} rank(s) (mums_shard_run)",
                       "rank0_phase_ms": {k: round(sm[k], 3) for k in ("ms_chains", "ms_replay", "ms_output")},
                       "ranks_chain_stage": ranks_chain,
                       "exchange": ("RCCL communicator inside libmums_hip.so (ncclCommInitRank): grouped "
                                    "ncclSend/ncclRecv all-to-allv, ncclAllGather of counts" if args.exchange == "abi"
                                    else f"torch.distributed {args.dist_backend} all_to_all (shard.py)")}
        except Exception as e:  # report, never hide
            mums_c3 = {"error": str(e)}
    seedmers_total = sum(max(n - lm.getSeedLength(seed) + 1, 0) for _ in range(G))
    seedmers_rank = st["seedmers"]
    key_bytes = st["key_bytes"]
    probes = st["probes"]
    if sharded and hasattr(stage, "close"):
        stage.close()
    mh.close()
    del genomes

    if rank == 0:
        value = seedmers_total * args.steps / dt
        achieved = bytes_dom / (ms_dom * 1e-3) / 1e9 if ms_dom > 0 else None
        traffic = None
        traffic_src = None
        # PMC counters cannot be read inside this run: the figure is the committed rocprofv3
        # FETCH_SIZE/WRITE_SIZE summary of the same kernel on the default N=1 workload
        if world == 1 and (G, n) == (8, 100_000_000) and os.path.exists(PROFILE_SUMMARY):
            try:
                traffic = json.load(open(PROFILE_SUMMARY)).get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(PROFILE_SUMMARY, ROOT) + " (rocprofv3 PMC passes, not this run)"
            except Exception:
                traffic = None
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "seed-mers/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",   # the C3 input is fixed and split over the ranks
            "vs_baseline": None,
            "dtype": "u64" if key_bytes == 8 else "u32",
            "data": (f"synthetic: {G} related genomes generated on the GPU (iid ACGT base, 1% substitutions"
                     + (", genome 2 reverse-complemented)" if G >= 3 else ")")),
            "config": {"workload": f"BASELINE config {5 if args.workload == 'c5' else 3}: {G} x {n // 10**6} Mbp, "
                                   f"seed weight 19 (0x7b974ef), MemHash seed stage (sorted+matched)"
                                   + (f", {st.get('chunks', 0)} key chunks" if world == 1 and args.workload == 'c5'
                                      else ""),
                       "genomes": G, "genome_length": n, "seedmers_total": seedmers_total,
                       "seedmers_rank0": seedmers_rank, "probes_rank0": probes,
                       "parallelism": (f"genome-sharded x{world}: "
                                       f"{'position slice' if args.workload == 'c5' else 'genome block'} per rank, "
                                       + (f"RCCL all-to-allv of key ranges inside libmums_hip.so (mums_shard_run, "
                                          f"ncclCommInitRank communicator), merge per key range"
                                          if args.exchange == "abi" else
                                          f"{'RCCL' if args.dist_backend == 'nccl' else args.dist_backend} all-to-all "
                                          f"of key ranges ({exch_bytes / max(args.steps, 1) / 1e9:.2f} GB/step sent by "
                                          f"rank 0), merge per key range")) if world > 1 else "1 GPU"},
            "roofline": {
                "bound": "hbm",
                "kernel": f"seg_onesweep_kernel (segmented onesweep LSD pass over packed 8-B seed records, "
                          f"{launches // max(args.steps, 1)} passes/step)",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "bytes_per_launch": bytes_dom / max(launches, 1),
                "avg_launch_ms": ms_dom / max(launches, 1),
                "timing": "HIP events around each launch on the context's stream, in K profiled steps run "
                          "after the timed region",
            },
            "phase_ms_per_step": {k: round(v / args.steps, 3) for k, v in phase.items()},
        }
        if mums_c3 is not None:
            out["mums_c3"] = mums_c3
        if e2e_c3 is not None:
            out["e2e_c3"] = e2e_c3
        if compat_c3 is not None:
            out["mums_c3_compat"] = compat_c3
        if fallback is not None:
            out["exchange_fallback"] = fallback + " -> torch.distributed RCCL all_to_all (libmems_amd/shard.py)"
        if not args.no_mums:
            progress("MUMs/s small configs")
            try:
                out["mums"] = run_mums(local, dev, 0.01)
                out["mums_iid"] = run_mums(local, dev, 1.0)
            except Exception as e:  # report, never hide
                out["mums"] = {"error": str(e)}
        if not args.no_cpu_baseline and world == 1:
            progress("CPU baselines")
            out["cpu_baseline"] = cpu_baseline()
            if not args.no_mums:
                out["cpu_baseline_mums"] = cpu_baseline_mums()
        progress("done")
        print(json.dumps(out), flush=True)
    if world > 1:
        barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
