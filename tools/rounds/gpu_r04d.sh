#!/bin/bash
# round 4: stream-built line rows (batched group loads) + onesweep line sort -- parity subset,
# A/B vs key-order rows and vs the 64-bit pair radix line sort, kernel trace
set -o pipefail
bash tools/gpu_tests.sh r04d tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_compat.py \
  tests/test_gpu_many_genomes.py tests/test_gpu_match_log.py tests/test_gpu_find_chunked.py || exit $?
for rep in 1 2; do
  echo "default:"; timeout -k 10 120 python3 -u tools/c3_mums.py 3 2>&1 | grep iter || exit 13
  echo "key rows:"; MUMS_DEV_KEY_ROWS=1 timeout -k 10 120 python3 -u tools/c3_mums.py 3 2>&1 | grep iter || exit 14
  echo "pair radix line sort:"; MUMS_DEV_LINE_RADIX=1 timeout -k 10 120 python3 -u tools/c3_mums.py 3 2>&1 | grep iter || exit 15
done
bash tools/prof_c3_mums.sh r04d_c3mums | tail -32
