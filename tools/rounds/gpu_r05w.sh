#!/bin/bash
# round 5: walk kernels' occupancy (MUMS_HIT_BATCH=1 and / or amdgpu_waves_per_eu(4)) vs the
# default build, C3 FindMatches, two repetitions (tools/rounds/ab_c3mums.sh)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05w
bash tools/rounds/ab_c3mums.sh default libmems_amd/var/libmums_b4.so libmems_amd/var/libmums_b2w4.so libmems_amd/var/libmums_b1.so 2>&1 | tee gpurun_out/r05w/ab3.txt
