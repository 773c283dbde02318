#!/bin/bash
# Sharded kept-probe export: the sharded suites
set -o pipefail
OUT=gpurun_out/r06h
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shard_abi.py tests/test_gpu_shard.py \
  tests/test_gpu_shard_restart.py tests/test_gpu_cpp_host.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 13; }
tail -3 $OUT/pytest.log
