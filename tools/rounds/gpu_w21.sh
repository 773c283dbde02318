#!/bin/bash
# One GPU call: w20-21 parity tests, w21 vs w19 seed-stage timing (split and one-level
# scatter), then onesweep knob variants A/B.   tools/gpu_w21.sh <tag> [variant libs...]
set -o pipefail
T=${1:-w21}; shift
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_w21.py tests/test_gpu_parity.py -m gpu -q -x -rf --timeout 200 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 11; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u tools/seed_patterns_bench.py --patterns 21:0,19:0 --tag split > $OUT/pat.jsonl 2> $OUT/pat.err || { tail -5 $OUT/pat.err; exit 12; }
MUMS_DEV_NO_SPLIT=1 timeout -k 10 200 python -u tools/seed_patterns_bench.py --patterns 21:0 --tag onelevel >> $OUT/pat.jsonl 2>> $OUT/pat.err || { tail -5 $OUT/pat.err; exit 13; }
cat $OUT/pat.jsonl
[ $# -gt 0 ] && bash tools/ab.sh ${T}_ab "$@"
exit 0
