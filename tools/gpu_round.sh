#!/bin/bash
# One GPU call: parity tests, smoke, bench (N=1).  Outputs under gpurun_out/<tag>/.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed $?"; tail -30 $OUT/pytest_gpu.log; exit 11; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $OUT/smoke.log; exit 12; }
cat $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 13; }
cat $OUT/bench.json
