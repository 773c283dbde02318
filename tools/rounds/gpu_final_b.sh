#!/bin/bash
# round evidence, part B: PMC passes of every FindMatches chain / replay kernel on C3, and the
# N-gapped config-5 FindMatches at w21 (two calls)
set -o pipefail
T=${1:-r03h}
bash tools/pmc_chains.sh ${T}_pmc_chains || exit $?
mkdir -p gpurun_out/$T
MUMS_DEV_RESTART_TIMING=1 timeout -k 10 500 python -u tools/bench_c5.py --weight 21 --gaps 100 --steps 1 --find-steps 2 > gpurun_out/$T/c5_w21_gaps.log 2>&1 || { tail -20 gpurun_out/$T/c5_w21_gaps.log; exit 31; }
grep -v "tie replay level" gpurun_out/$T/c5_w21_gaps.log | tail -14
