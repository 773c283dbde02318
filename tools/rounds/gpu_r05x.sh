#!/bin/bash
# round 5: hit_word's window loads as one 16-B + one 12-B load per genome (default) vs one
# load per word (MUMS_HIT_VEC=0 build): walk parity tests, then C3 FindMatches A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05x
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_walk_refill.py tests/test_gpu_row_paths.py tests/test_gpu_parity.py > gpurun_out/r05x/pytest.log 2>&1 || { tail -30 gpurun_out/r05x/pytest.log; exit 11; }
tail -2 gpurun_out/r05x/pytest.log
bash tools/rounds/ab_c3mums.sh default libmems_amd/var/libmums_novec.so 2>&1 | tee gpurun_out/r05x/ab.txt
