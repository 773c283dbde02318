#!/bin/bash
# Persistent onesweep pass A/B: per-phase stats (stats builds) + same-box timing + parity under it.
set -o pipefail
OUT=gpurun_out/r06b
mkdir -p $OUT
for v in "osstats 1" "osstats_pf0 1"; do
  set -- $v
  MUMS_DEV_OS_PERSIST=$2 MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_$1.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-mums --no-cpu-baseline \
    > $OUT/stats_$1.json 2> $OUT/stats_$1.err || { tail -20 $OUT/stats_$1.err; exit 11; }
  echo "== $1 persist"; grep os_stats $OUT/stats_$1.err | tail -4
done
for rep in 1 2; do
  for v in "default 0" "default 1" "pf0 1"; do
    set -- $v
    if [ $1 = default ]; then unset MUMS_DEV_LIB; else export MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_$1.so; fi
    if [ $2 = 1 ]; then export MUMS_DEV_OS_PERSIST=1; else unset MUMS_DEV_OS_PERSIST; fi
    timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-mums --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 12; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$1 persist=$2', round(d['ms_per_step'],2), 'ms/step onesweep', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],3), d['phase_ms_per_step'])"
  done
done
unset MUMS_DEV_LIB
MUMS_DEV_OS_PERSIST=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_large.py \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 13; }
tail -3 $OUT/pytest.log
