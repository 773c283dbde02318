#!/bin/bash
# round 4: tie workspace kept as the chunked FindMatches arena -- restart / chunked tests, then the
# N-gapped config-5 w21 FindMatches (3 calls) with the restart phase timing
set -o pipefail
T=r04f
OUT=gpurun_out/$T
mkdir -p $OUT
bash tools/gpu_tests.sh $T tests/test_gpu_chunked_restart.py tests/test_gpu_find_chunked.py tests/test_gpu_chunked.py || exit $?
MUMS_DEV_RESTART_TIMING=1 timeout -k 10 600 python -u tools/bench_c5.py --weight 21 --gaps 100 --steps 1 --find-steps 3 > $OUT/c5.log 2>&1 || { tail -20 $OUT/c5.log; exit 12; }
grep -E "restart phase tie workspace|FindMatches [0-9]|step " $OUT/c5.log | tail -14
tail -1 $OUT/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['findmatches']; print('seed ms/step', d['ms_per_step'], 'find ms', f['ms'], f['matches'], f['phase_ms'])"
