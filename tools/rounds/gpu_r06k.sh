#!/bin/bash
# Sharded kept-probe export after the communicator copy-ordering fix: C3 over 4 in-process ranks + the sharded suites
set -o pipefail
OUT=gpurun_out/r06k
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/dev/shard_exchange_c3.py 4 > $OUT/shard_exchange_c3_w4.txt 2>&1 || { tail -20 $OUT/shard_exchange_c3_w4.txt; exit 11; }
cat $OUT/shard_exchange_c3_w4.txt
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_shard_abi.py tests/test_gpu_shard.py \
  tests/test_gpu_shard_restart.py tests/test_gpu_compat_ranks.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 13; }
tail -2 $OUT/pytest.log
