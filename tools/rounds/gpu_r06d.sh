#!/bin/bash
# Multi-tile onesweep blocks A/B (MUMS_DEV_OS_PERSIST 0 / 4 = 1 tile, 2 = 2 tiles, 3 = 4 tiles, 1 = persistent)
set -o pipefail
OUT=gpurun_out/r06d
mkdir -p $OUT
for v in 4 2 3; do
  MUMS_DEV_OS_PERSIST=$v MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_osstats.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-mums --no-cpu-baseline \
    > $OUT/stats_$v.json 2> $OUT/stats_$v.err || { tail -20 $OUT/stats_$v.err; exit 11; }
  echo "== stats persist=$v"; grep os_stats $OUT/stats_$v.err | tail -2
done
for rep in 1 2; do
  for v in 0 2 3 1; do
    if [ $v = 0 ]; then unset MUMS_DEV_OS_PERSIST; else export MUMS_DEV_OS_PERSIST=$v; fi
    timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-mums --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 12; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']
print('persist=$v', round(d['ms_per_step'],2), 'ms/step onesweep', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],3), d['phase_ms_per_step'])"
  done
done
unset MUMS_DEV_OS_PERSIST
MUMS_DEV_OS_PERSIST=2 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_large.py \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 13; }
tail -1 $OUT/pytest.log
