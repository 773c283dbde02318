#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04p
export MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_lh16.so
timeout -k 10 120 python -u tools/c3_mums.py 1 2>&1 | grep -v amdgpu.ids | tail -5
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 2>&1 | grep -E "Error|assert|FAILED|passed|failed" | head -12
export MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_lh24.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_find_chunked.py -m gpu -q -x --timeout 200 2>&1 | grep -E "Error|assert|FAILED|passed|failed" | head -12
