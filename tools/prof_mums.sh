#!/bin/bash
# rocprofv3 kernel trace of one FindMatches on the BASELINE config-2 shape (run via gpurun)
set -o pipefail
T=${1:-mums}
export TMPDIR=/tmp
mkdir -p gpurun_out/$T
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/kt -o kt -- python3 tools/replay_dbg.py > gpurun_out/$T/kt.log 2>&1 || { tail -20 gpurun_out/$T/kt.log; exit 11; }
tail -3 gpurun_out/$T/kt.log
python3 - <<PY
import csv
r = list(csv.DictReader(open("gpurun_out/$T/kt/kt_kernel_stats.csv")))
for x in r[:25]:
    print(f"{float(x['TotalDurationNs'])/1e6/2:9.3f} ms/iter {int(x['Calls'])//2:5d} calls  {x['Name'][:110]}")
PY
