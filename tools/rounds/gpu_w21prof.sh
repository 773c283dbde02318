#!/bin/bash
# w21 seed stage: parity tests, timing (split vs one-level), kernel trace of the split path.
set -o pipefail
T=${1:-w21p}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_w21.py -m gpu -q -x -rf --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 11; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u tools/seed_patterns_bench.py --patterns 21:0,19:0 --tag split > $OUT/pat.jsonl 2> $OUT/pat.err || { tail -5 $OUT/pat.err; exit 12; }
cat $OUT/pat.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 -u tools/seed_patterns_bench.py --patterns 21:0 --steps 2 > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 13; }
python3 - <<PY
import csv
r = list(csv.DictReader(open("$OUT/kt/kt_kernel_stats.csv")))
for x in r[:16]:
    print(f"{float(x['AverageNs'])/1e3:10.1f} us avg {int(x['Calls']):4d} calls  {x['Name'][:110]}")
PY
