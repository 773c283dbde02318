#!/bin/bash
# round evidence, part A: the whole -m gpu suite, smoke, bench (N=1), rocprofv3 kernel trace +
# FETCH/WRITE passes of the bench, kernel trace of C3 FindMatches
set -o pipefail
T=${1:-r03g}
bash tools/gpu_round.sh $T || exit $?
bash tools/profile_round.sh $T || exit $?
bash tools/prof_c3_mums.sh ${T}_c3mums > /dev/null || exit 21
echo done
