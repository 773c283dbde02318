#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04k
MUMS_DEV_SHARD_RESTART_DEBUG=1 timeout -k 10 120 python -u tools/dbg_shard_restart.py 2>&1 | grep -v amdgpu.ids
