"""Copy a GPU evidence run (tools/rounds/gpu_r06*.sh + tools/round_evidence.sh) from gpurun_out/
into profiles/ under its tag:  python tools/save_evidence.py <run> <ev_tag> [note]
  <run>     gpurun_out/<run>/{pytest.log, smoke.log}  -> profiles/<run>_pytest_gpu_tail.log, _smoke.log
  <ev_tag>  gpurun_out/<ev_tag>/ (kernel trace + PMC passes + bench) -> tools/summarize_profile.py,
            profiles/<ev_tag>_bench.json; gpurun_out/<ev_tag>_c3/ -> profiles/<ev_tag>_c3_findmatches_*"""
import csv
import os
import shutil
import subprocess
import sys

run, tag = sys.argv[1], sys.argv[2]
note = sys.argv[3] if len(sys.argv) > 3 else ""
src, dst = os.path.join("gpurun_out", run), "profiles"
for name, out in (("pytest.log", "pytest_gpu_tail.log"), ("smoke.log", "smoke.log")):
    p = os.path.join(src, name)
    if os.path.exists(p):
        lines = open(p).read().splitlines()
        open(os.path.join(dst, f"{run}_{out}"), "w").write("\n".join(lines[-15:]) + "\n")
subprocess.run([sys.executable, "tools/summarize_profile.py", tag], check=True)
bench = [l for l in open(os.path.join("gpurun_out", tag, "bench.json")).read().splitlines()
         if l.startswith('{"metric"')]
open(os.path.join(dst, f"{tag}_bench.json"), "w").write(bench[-1] + "\n")
c3 = os.path.join("gpurun_out", f"{tag}_c3")
if os.path.isdir(c3):
    rows = list(csv.DictReader(open(os.path.join(c3, "kt", "kt_kernel_stats.csv"))))
    lines = [f"# C3 FindMatches kernel trace ({note + ', ' if note else ''}`tools/prof_c3_mums.sh`: tools/c3_mums.py 2 = "
             "two FindMatches calls, ms per call = total / 2; the `at::native` kernels build the synthetic input)", "",
             "| kernel | calls | total ms | ms per FindMatches | avg us |", "|---|---|---|---|---|"]
    for r in rows[:40]:
        tot = float(r["TotalDurationNs"]) / 1e6
        lines.append(f"| `{r['Name'][:100]}` | {r['Calls']} | {tot:.3f} | {tot / 2:.3f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} |")
    open(os.path.join(dst, f"{tag}_c3_findmatches_kernel_stats.md"), "w").write("\n".join(lines) + "\n")
    shutil.copy(os.path.join(c3, "plain.log"), os.path.join(dst, f"{tag}_c3_findmatches_plain.log"))
print("saved", run, tag)
