#!/bin/bash
# round 5: the hash sort's digit histograms counted by line_rec2_kernel (default) vs the
# histogram read of its records (MUMS_DEV_LINE_GHIST=1): parity, then C3 alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z4
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_walk_refill.py tests/test_gpu_row_paths.py tests/test_gpu_large.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py > gpurun_out/r05z4/pytest.log 2>&1 || { tail -30 gpurun_out/r05z4/pytest.log; exit 11; }
tail -2 gpurun_out/r05z4/pytest.log
for rep in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export MUMS_DEV_LINE_GHIST=1; else unset MUMS_DEV_LINE_GHIST; fi
    echo "line_ghist=$v: $(timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" | tee -a gpurun_out/r05z4/ab.txt
  done
done
