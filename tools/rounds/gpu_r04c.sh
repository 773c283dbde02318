#!/bin/bash
# round 4: FindMatches with rows built from the stream in line order -- parity, then A/B vs key-order rows
set -o pipefail
bash tools/gpu_tests.sh r04c tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_compat.py \
  tests/test_gpu_many_genomes.py tests/test_gpu_restart.py tests/test_gpu_match_log.py tests/test_gpu_sweep.py || exit $?
for rep in 1 2; do
  echo "stream rows:"; timeout -k 10 120 python3 -u tools/c3_mums.py 3 2>&1 | grep iter || exit 13
  echo "key rows:"; MUMS_DEV_KEY_ROWS=1 timeout -k 10 120 python3 -u tools/c3_mums.py 3 2>&1 | grep iter || exit 14
done
bash tools/prof_c3_mums.sh r04c_c3mums | tail -32
