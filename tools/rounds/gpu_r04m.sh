#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04m
timeout -k 10 400 python -u tools/bench_shard_restart.py --length 100000000 --gaps 100 --world 8 > gpurun_out/r04m/shard_restart.log 2>&1 || { tail -20 gpurun_out/r04m/shard_restart.log; exit 3; }
grep -v amdgpu.ids gpurun_out/r04m/shard_restart.log
