#!/bin/bash
# Probe stage with the look-back (probes at their final offsets, no probe_compact) A/B + parity
set -o pipefail
OUT=gpurun_out/${1:-r06v}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_restart.py tests/test_gpu_compat.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 11; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for v in lb compact; do
    if [ $v = compact ]; then export MUMS_DEV_PROBE_COMPACT=1; else unset MUMS_DEV_PROBE_COMPACT; fi
    timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 12; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', round(d['ms_per_step'],2), 'ms/step onesweep', round(r['avg_launch_ms'],3), d['phase_ms_per_step'], 'C3 find', round(d['mums_c3']['ms'],2), 'compat', round(d['mums_c3_compat']['ms'],2))"
  done
done
unset MUMS_DEV_PROBE_COMPACT
