#!/bin/bash
# round 5: the chains' (bucket, block) sort on bucket + block-key bits (3 passes at C3) vs
# 64 bits (8 passes; var/libmums_g64.so = the previous replay.hip): parity, then C3 A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_many_genomes.py tests/test_gpu_compat.py tests/test_gpu_shard_abi.py > gpurun_out/r05z1/pytest.log 2>&1 || { tail -30 gpurun_out/r05z1/pytest.log; exit 11; }
tail -2 gpurun_out/r05z1/pytest.log
bash tools/rounds/ab_c3mums.sh default libmems_amd/var/libmums_g64.so 2>&1 | tee gpurun_out/r05z1/ab.txt
