#!/bin/bash
# tie workspace kept across seed-stage-only chunked calls: restart tests, then config-5
# N-gapped w21 (3 seed-stage steps + 1 FindMatches) with the restart phase timing
set -o pipefail
T=${1:-r03r}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_chunked_restart.py tests/test_gpu_restart.py tests/test_gpu_progress.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 11; }
tail -1 $OUT/pytest.log
MUMS_DEV_RESTART_TIMING=1 timeout -k 10 500 python -u tools/bench_c5.py --weight 21 --gaps 100 --steps 3 --find-steps 1 > $OUT/c5.log 2>&1 || { tail -20 $OUT/c5.log; exit 12; }
grep -E "restart phase tie workspace|FindMatches [0-9]" $OUT/c5.log | tail -12
tail -1 $OUT/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('seed ms/step', d['ms_per_step'], 'find ms', d['findmatches']['ms'], d['findmatches']['matches'])"
