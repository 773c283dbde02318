#!/bin/bash
# sharded restart at scale: 2 x 1 Gbp N-gapped, w21, 33-bit records, 8 ranks on one GPU
set -o pipefail
mkdir -p gpurun_out/r04n
MUMS_DEV_SHARD_IB33=1 timeout -k 10 900 python -u tools/bench_shard_restart.py --length 500000000 --gaps 200 --world 8 --weight 21 --modes local,gather 2>&1 | tee gpurun_out/r04n/shard_restart.log || { tail -20 gpurun_out/r04n/shard_restart.log; exit 3; }
