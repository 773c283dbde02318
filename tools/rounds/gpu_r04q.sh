#!/bin/bash
# line-hash collisions: detection + exact line order (16-bit hash forces collisions)
set -o pipefail
mkdir -p gpurun_out/r04q
echo "default C3:"; MUMS_DEV_CHAIN_DEBUG=1 timeout -k 10 120 python -u tools/c3_mums.py 2 2>&1 | grep -E "collision|iter" | tail -3
export MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_lh16.so
echo "16-bit hash C3:"; MUMS_DEV_CHAIN_DEBUG=1 timeout -k 10 120 python -u tools/c3_mums.py 1 2>&1 | grep -E "collision|iter" | tail -3
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_find_chunked.py -m gpu -q -x --timeout 200 2>&1 | grep -E "Error|assert|FAILED|passed|failed" | head -8
unset MUMS_DEV_LIB
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py -m gpu -q -x --timeout 200 2>&1 | grep -E "Error|assert|FAILED|passed|failed" | head -8
