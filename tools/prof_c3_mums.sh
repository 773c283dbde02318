#!/bin/bash
# rocprofv3 kernel trace of full FindMatches on BASELINE config 3 (run via gpurun)
set -o pipefail
T=${1:-c3mums}
export TMPDIR=/tmp
mkdir -p gpurun_out/$T
timeout -k 10 120 env MUMS_DEV_CHAIN_DEBUG=1 python3 -u tools/c3_mums.py 2 > gpurun_out/$T/plain.log 2>&1 || { tail -20 gpurun_out/$T/plain.log; exit 10; }
cat gpurun_out/$T/plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/kt -o kt -- python3 -u tools/c3_mums.py 2 > gpurun_out/$T/kt.log 2>&1 || { tail -20 gpurun_out/$T/kt.log; exit 11; }
python3 - <<PY
import csv
r = list(csv.DictReader(open("gpurun_out/$T/kt/kt_kernel_stats.csv")))
for x in r[:30]:
    print(f"{float(x['TotalDurationNs'])/1e6/3:9.3f} ms/iter {int(x['Calls'])//3:5d} calls avg {float(x['AverageNs'])/1e3:9.1f} us  {x['Name'][:100]}")
PY
