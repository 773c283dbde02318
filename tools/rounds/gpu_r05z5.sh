#!/bin/bash
# round 5: the line order stored by the hash sort's last pass (default) vs the records + line_ord_kernel (MUMS_DEV_LINE_ORD=1); segment flags from chain_left_kernel
# (both runs): parity, then C3 alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z5
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_walk_refill.py tests/test_gpu_row_paths.py tests/test_gpu_large.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py tests/test_gpu_compat.py tests/test_gpu_chunked.py > gpurun_out/r05z5/pytest.log 2>&1 || { tail -30 gpurun_out/r05z5/pytest.log; exit 11; }
tail -2 gpurun_out/r05z5/pytest.log
for rep in 1 2; do
  for v in 0 1; do
    if [ $v = 1 ]; then export MUMS_DEV_LINE_ORD=1; else unset MUMS_DEV_LINE_ORD; fi
    echo "line_ord_kernel=$v: $(timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" | tee -a gpurun_out/r05z5/ab.txt
  done
done
# the materialize kernel's 16-B record loads (default) vs 8-B (MUMS_MAT_WIDE=0 build)
bash tools/rounds/ab_c3mums.sh default libmems_amd/var/libmums_matnarrow.so 2>&1 | tee gpurun_out/r05z5/ab_mat.txt
