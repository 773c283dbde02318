#!/bin/bash
set -o pipefail
OUT=gpurun_out/r06g
mkdir -p $OUT
VAR=MUMS_DEV_PROBE_GENERAL VALS="1 0" bash tools/ab_env.sh r06g_ab || exit 12
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_many_genomes.py tests/test_gpu_restart.py \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 14; }
tail -1 $OUT/pytest.log
