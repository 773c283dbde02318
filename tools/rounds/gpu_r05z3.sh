#!/bin/bash
# round 5: FindMatches without the bucket order of all probes (the replay orders its kept
# probes itself) vs with it (MUMS_DEV_KEEP_BUCKET_ORDER=1): parity, then C3 alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z3
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_compat.py tests/test_gpu_large.py tests/test_gpu_find_chunked.py tests/test_gpu_compat_logs.py tests/test_gpu_many_genomes.py tests/test_gpu_result_out.py tests/test_gpu_replay_big.py tests/test_gpu_match_log.py tests/test_gpu_restart.py > gpurun_out/r05z3/pytest.log 2>&1 || { tail -30 gpurun_out/r05z3/pytest.log; exit 11; }
tail -2 gpurun_out/r05z3/pytest.log
for rep in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export MUMS_DEV_KEEP_BUCKET_ORDER=1; else unset MUMS_DEV_KEEP_BUCKET_ORDER; fi
    echo "keep_order=$v: $(timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" | tee -a gpurun_out/r05z3/ab.txt
  done
done
