#!/bin/bash
set -o pipefail
T=${1:-r03f}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tie_order.py tests/test_gpu_restart.py tests/test_gpu_overlaps.py \
  tests/test_gpu_chunked_restart.py tests/test_gpu_shard_restart.py tests/test_gpu_enumerate.py -m gpu -v -x -rf --timeout 200 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 11; }
tail -1 $OUT/pytest.log
MUMS_DEV_RESTART_TIMING=1 timeout -k 10 400 python -u tools/bench_c5.py --weight 21 --gaps 100 --steps 2 --find-steps 1 > $OUT/c5_w21_gaps.log 2>&1 || { tail -20 $OUT/c5_w21_gaps.log; exit 12; }
grep -v "tie replay level" $OUT/c5_w21_gaps.log | tail -12
