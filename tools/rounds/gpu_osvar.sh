#!/bin/bash
# A/B of the onesweep block shapes (MUMS_DEV_OS_VARIANT, radix_seg.hip) inside one call:
# bit-exact check of every variant on the parity inputs, then the C3 seed-stage bench.
set -o pipefail
T=${1:-r03j}
OUT=gpurun_out/$T
mkdir -p $OUT
for v in ${VARS:-1 2 4 5}; do
  MUMS_DEV_OS_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_w21.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > $OUT/pytest_v$v.log 2>&1 || { echo "variant $v failed"; tail -30 $OUT/pytest_v$v.log; exit 11; }
  echo "variant $v: $(tail -1 $OUT/pytest_v$v.log)"
done
for rep in 1 2; do
  for v in ${BVARS:-0 1 2 4 5}; do
    MUMS_DEV_OS_VARIANT=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-mums > $OUT/bench_v${v}_$rep.json 2> $OUT/bench_v${v}_$rep.err || { echo "bench $v failed"; tail -20 $OUT/bench_v${v}_$rep.err; exit 12; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_v${v}_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('v$v', d['ms_per_step'], r['achieved'], r['frac'], d.get('phase_ms', d.get('config',{}).get('phase_ms')))"
  done
done
