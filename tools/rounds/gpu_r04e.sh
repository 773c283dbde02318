#!/bin/bash
# round 4: fused materialize (line keys + first starts), LDS-staged row gather, onesweep line sort
set -o pipefail
timeout -k 10 120 python3 -u tools/dbg_r04.py 2>&1 | grep -v amdgpu.ids || exit 9
bash tools/gpu_tests.sh r04e tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_compat.py \
  tests/test_gpu_many_genomes.py tests/test_gpu_match_log.py tests/test_gpu_find_chunked.py tests/test_gpu_restart.py \
  tests/test_gpu_enumerate.py tests/test_gpu_pairwise.py || exit $?
for rep in 1 2; do
  echo "default:"; timeout -k 10 120 python3 -u tools/c3_mums.py 3 2>&1 | grep iter || exit 13
  echo "pair radix line sort:"; MUMS_DEV_LINE_RADIX=1 timeout -k 10 120 python3 -u tools/c3_mums.py 3 2>&1 | grep iter || exit 15
done
bash tools/prof_c3_mums.sh r04e_c3mums | tail -32
