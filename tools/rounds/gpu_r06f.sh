#!/bin/bash
# Probe stage: compile-time default-tolerance kernel (fewer SGPR spills) A/B + PMC of the seed kernels
set -o pipefail
OUT=gpurun_out/r06f
mkdir -p $OUT
VAR=MUMS_DEV_PROBE_GENERAL VALS="1 0" bash tools/ab_env.sh r06f_ab || exit 12
NO_YARDSTICK=1 bash tools/pmc_onesweep.sh r06f_pmc > $OUT/pmc.txt 2>&1 || { tail -20 $OUT/pmc.txt; exit 13; }
grep -E "probe_tile|seed_scatter" $OUT/pmc.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_many_genomes.py \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 14; }
tail -1 $OUT/pytest.log
