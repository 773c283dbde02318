#!/bin/bash
# Claim descriptors in the XCD queues (MUMS_DEV_OS_XD) A/B + stats + parity
set -o pipefail
OUT=gpurun_out/r06e
mkdir -p $OUT
for v in 0 1; do
  MUMS_DEV_OS_XD=$v MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_osstats.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-mums --no-cpu-baseline \
    > $OUT/stats_$v.json 2> $OUT/stats_$v.err || { tail -20 $OUT/stats_$v.err; exit 11; }
  echo "== stats xd=$v"; grep os_stats $OUT/stats_$v.err | tail -2
done
VAR=MUMS_DEV_OS_XD VALS="0 1" bash tools/ab_env.sh r06e_ab || exit 12
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_compat.py \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 13; }
tail -1 $OUT/pytest.log
