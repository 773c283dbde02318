#!/bin/bash
# round 4 evidence: rocprofv3 kernel trace + FETCH / WRITE passes of the bench seed stage,
# kernel trace of C3 FindMatches, FETCH / WRITE of the C3 FindMatches chain kernels
set -o pipefail
T=r04l
bash tools/profile_round.sh $T || exit $?
bash tools/prof_c3_mums.sh ${T}_c3mums | tail -32 || exit 21
