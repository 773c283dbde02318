#!/bin/bash
# Round evidence on the GPU box: rocprofv3 kernel trace + FETCH/WRITE passes of the bench
# (seed stage), kernel trace of the C3 FindMatches, full bench line.
set -o pipefail
TAG=${1:-r01}
bash tools/profile_round.sh $TAG || exit $?
bash tools/prof_c3_mums.sh ${TAG}_c3 > /dev/null || exit 21
timeout -k 10 600 python3 -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -5 gpurun_out/$TAG/bench.err; exit 22; }
cat gpurun_out/$TAG/bench.json
