#!/bin/bash
# the rest of r03b (multi-process ABI slices case, w21 profile) + the parity subset and C3 FindMatches timing
set -o pipefail
T=${1:-r03c}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_pairwise.py tests/test_gpu_enumerate.py tests/test_gpu_compat.py tests/test_gpu_shard.py -k "abi_multiprocess or pairwise or enum or compat or Pairwise or Parallel" -m gpu -q -x -rf --timeout 300 \
  --timeout-method thread > $OUT/pytest_mp.log 2>&1 || { echo "pytest mp failed"; tail -30 $OUT/pytest_mp.log; exit 11; }
tail -1 $OUT/pytest_mp.log
bash tools/gpu_quick.sh ${T}_quick || exit 12
timeout -k 10 200 python -u tools/seed_patterns_bench.py --patterns 21:0,19:0 --tag split > $OUT/pat.jsonl 2> $OUT/pat.err || { tail -5 $OUT/pat.err; exit 13; }
cat $OUT/pat.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 -u tools/seed_patterns_bench.py --patterns 21:0 --steps 2 > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 14; }
python3 - <<PY
import csv
r = list(csv.DictReader(open("$OUT/kt/kt_kernel_stats.csv")))
for x in r[:16]:
    print(f"{float(x['AverageNs'])/1e3:10.1f} us avg {int(x['Calls']):4d} calls  {x['Name'][:110]}")
PY
