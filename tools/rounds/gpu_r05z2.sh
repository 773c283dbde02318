#!/bin/bash
# round 5: chain_link with the row loads of 4 (default) / 8 items in flight together vs one
# at a time (MUMS_LINK_PRE=1 build): parity, then C3 A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z2
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_walk_refill.py tests/test_gpu_row_paths.py tests/test_gpu_parity.py > gpurun_out/r05z2/pytest.log 2>&1 || { tail -30 gpurun_out/r05z2/pytest.log; exit 11; }
tail -2 gpurun_out/r05z2/pytest.log
bash tools/rounds/ab_c3mums.sh default libmems_amd/var/libmums_pre1.so libmems_amd/var/libmums_pre8.so 2>&1 | tee gpurun_out/r05z2/ab.txt
