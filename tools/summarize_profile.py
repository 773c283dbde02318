"""Summarize a rocprofv3 round profile (kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes)
into profiles/<tag>_*.  Dominant kernel = seg_onesweep_kernel (one LSD pass of the
segmented seed-record sort, 4 launches per step for w19).
HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE/WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE counts half of a wide streaming read (MI355X_MICROARCH.md "HBM"),
so it is doubled; this correction is calibrated for 16-B/lane streams only (the record loads
are 8 B/lane), so the traffic figure is reported with that caveat."""
import csv, json, os, sys, collections

DOM = "seg_onesweep_kernel"

tag = sys.argv[1]
src = os.path.join("gpurun_out", tag)
dst = "profiles"
os.makedirs(dst, exist_ok=True)
stats = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
lines = ["| kernel | calls | total ms | avg ms | % |", "|---|---|---|---|---|"]
for r in stats:
    lines.append(f"| `{r['Name'][:110]}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.3f} | "
                 f"{float(r['AverageNs'])/1e6:.3f} | {float(r['Percentage']):.2f} |")
open(os.path.join(dst, f"{tag}_kernel_stats.md"), "w").write("\n".join(lines) + "\n")

def pmc(name):
    d = collections.defaultdict(list)
    p = os.path.join(src, name, "pmc_counter_collection.csv")
    if not os.path.exists(p):
        return d
    for r in csv.DictReader(open(p)):
        d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return d

fetch, write = pmc("pmc_fetch"), pmc("pmc_write")
out = {"tag": tag, "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    if "mums::" not in k:
        continue
    f = fetch.get(k, []); w = write.get(k, [])
    out["kernels"][k[:120]] = {"launches": len(f), "fetch_kib_avg": sum(f)/len(f) if f else None,
                               "write_kib_avg": sum(w)/len(w) if w else None}
tot_f = sum(sum(fetch[k2]) for k2 in fetch if DOM in k2)
tot_w = sum(sum(write[k2]) for k2 in write if DOM in k2)
nl = sum(len(fetch[k2]) for k2 in fetch if DOM in k2)
ktd = [r for r in stats if DOM in r["Name"]]
calls = sum(int(r["Calls"]) for r in ktd); tot_ns = sum(float(r["TotalDurationNs"]) for r in ktd)
out["dominant_kernel"] = DOM
out["kernel_trace_avg_ms"] = tot_ns / calls / 1e6 if calls else None
out["kernel_trace_calls"] = calls
if nl:
    out["fetch_kib_per_launch"] = tot_f / nl
    out["write_kib_per_launch"] = tot_w / nl
    out["hbm_bytes_per_launch"] = (2 * tot_f + tot_w) / nl * 1024
    out["hbm_bytes_per_launch_uncorrected"] = (tot_f + tot_w) / nl * 1024
bench = [l for l in open(os.path.join(src, "kt.log")).read().splitlines() if l.startswith('{"metric"')]
if bench:
    open(os.path.join(dst, f"{tag}_bench_profiled.json"), "w").write(bench[-1] + "\n")
json.dump(out, open(os.path.join(dst, f"{tag}_dominant_kernel.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))
