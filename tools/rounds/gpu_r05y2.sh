#!/bin/bash
# round 5: long walks sharing window words across the lane group (default, DPP row shifts) vs loading them (MUMS_GRP_WORDS=0 build)
# load per word (MUMS_HIT_VEC=0 build): walk parity tests, then C3 FindMatches A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05y3
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_walk_refill.py tests/test_gpu_row_paths.py tests/test_gpu_parity.py > gpurun_out/r05y3/pytest.log 2>&1 || { tail -30 gpurun_out/r05y3/pytest.log; exit 11; }
tail -2 gpurun_out/r05y3/pytest.log
bash tools/rounds/ab_c3mums.sh default libmems_amd/var/libmums_nogrp.so 2>&1 | tee gpurun_out/r05y3/ab.txt
