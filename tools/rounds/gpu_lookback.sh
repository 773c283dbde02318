#!/bin/bash
# A/B of the onesweep look-back window (MUMS_LOOKBACK 2 / 4 / 8 predecessor statuses per
# step; variants built as libmems_amd/var/libmums_lb*.so, loaded through MUMS_DEV_LIB)
set -o pipefail
T=${1:-r03u}
OUT=gpurun_out/$T
mkdir -p $OUT
for v in 2 8; do
  MUMS_DEV_LIB=libmems_amd/var/libmums_lb$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > $OUT/pytest_lb$v.log 2>&1 || { echo "lb$v failed"; tail -20 $OUT/pytest_lb$v.log; exit 11; }
  echo "lb$v: $(tail -1 $OUT/pytest_lb$v.log)"
done
for rep in 1 2; do
  for v in 4 2 8; do
    L=""; [ $v != 4 ] && L=libmems_amd/var/libmums_lb$v.so
    MUMS_DEV_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-mums > $OUT/bench_lb${v}_$rep.json 2> $OUT/bench_lb${v}_$rep.err || { tail -20 $OUT/bench_lb${v}_$rep.err; exit 12; }
    python3 -c "import json; d=json.loads(open('$OUT/bench_lb${v}_$rep.json').read().strip().splitlines()[-1]); print('lb$v', round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],4), d['phase_ms_per_step']['ms_sort'])"
  done
done
