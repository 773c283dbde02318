#!/bin/bash
# Direct compat records: parity (compat tests), C3 A/B against the partition path
set -o pipefail
OUT=gpurun_out/r06p
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_compat.py -k "direct" > $OUT/direct.log 2>&1 || { tail -40 $OUT/direct.log; exit 11; }
grep -a "compat direct\|passed\|failed" $OUT/direct.log | tail -30
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_compat.py tests/test_gpu_compat_logs.py tests/test_gpu_tie_order.py tests/test_gpu_compat_ranks.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 12; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
  MUMS_DEV_COMPAT_DEBUG=1 timeout -k 10 300 python3 -u tools/dev/compat_c3.py 3 > $OUT/c3_direct.log 2>&1 || { tail -20 $OUT/c3_direct.log; exit 13; }
  grep -a "iter\|compat direct" $OUT/c3_direct.log | tail -3
  MUMS_DEV_COMPAT_PART=1 timeout -k 10 300 python3 -u tools/dev/compat_c3.py 3 > $OUT/c3_part.log 2>&1 || { tail -20 $OUT/c3_part.log; exit 14; }
  grep -a "iter" $OUT/c3_part.log | tail -2
done
