#!/bin/bash
# >32-genome finders, the parity subset + C3 FindMatches timing (probe rows staged in LDS), then the
# paired-load onesweep A/B and the w21 seed-stage profile
set -o pipefail
T=${1:-r03d}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_many_genomes.py -m gpu -v -x -rf --timeout 200 --timeout-method thread \
  > $OUT/pytest_many.log 2>&1 || { echo "pytest many failed"; tail -30 $OUT/pytest_many.log; exit 11; }
tail -1 $OUT/pytest_many.log
bash tools/gpu_quick.sh ${T}_quick || exit 12
bash tools/gpu_pair.sh ${T}_pair || exit 13
timeout -k 10 200 python -u tools/seed_patterns_bench.py --patterns 21:0,19:0 --tag split > $OUT/pat.jsonl 2> $OUT/pat.err || { tail -5 $OUT/pat.err; exit 14; }
cat $OUT/pat.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 -u tools/seed_patterns_bench.py --patterns 21:0 --steps 2 > $OUT/kt.log 2>&1 || { tail -5 $OUT/kt.log; exit 15; }
python3 - <<PY
import csv
r = list(csv.DictReader(open("$OUT/kt/kt_kernel_stats.csv")))
for x in r[:16]:
    print(f"{float(x['AverageNs'])/1e3:10.1f} us avg {int(x['Calls']):4d} calls  {x['Name'][:110]}")
PY
