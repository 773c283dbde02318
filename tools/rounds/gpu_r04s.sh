#!/bin/bash
# line-order keep pass (no chain_of scatter): C3 timing + FindMatches parity files
set -o pipefail
for rep in 1 2; do
  echo "c3: $(timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" || exit 1
done
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py tests/test_gpu_replay_big.py tests/test_gpu_match_log.py tests/test_gpu_tie_order.py tests/test_gpu_restart.py tests/test_gpu_sweep.py tests/test_gpu_pairwise.py tests/test_gpu_enumerate.py tests/test_gpu_shard.py -m gpu -q -x --timeout 300 > gpurun_out/r04s_tests.log 2>&1; rc=$?
grep -E "Error|assert|FAILED|passed|failed" gpurun_out/r04s_tests.log | head -12
exit $rc
