#!/bin/bash
# long-walk handoff to whole waves: C3 timing (debug histogram once) + per-launch trace + parity
set -o pipefail
MUMS_DEV_CHAIN_DEBUG=1 timeout -k 10 120 python -u tools/c3_mums.py 1 2>&1 | grep -E "chains:|iter" || exit 1
for rep in 1 2; do
  echo "c3: $(timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" || exit 1
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04u_kt -o kt -- python3 -u tools/c3_mums.py 2 > gpurun_out/r04u_kt.log 2>&1 || exit 2
python3 - <<'PY'
import csv
r = list(csv.DictReader(open("gpurun_out/r04u_kt/kt_kernel_trace.csv")))
r.sort(key=lambda x: int(x['Start_Timestamp']))
print([(x['Kernel_Name'].split('(')[0].split('::')[-1][:26], round((int(x['End_Timestamp']) - int(x['Start_Timestamp'])) / 1e3))
       for x in r if 'chain_walk' in x['Kernel_Name']])
PY
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py tests/test_gpu_replay_big.py tests/test_gpu_match_log.py tests/test_gpu_tie_order.py tests/test_gpu_restart.py tests/test_gpu_sweep.py tests/test_gpu_pairwise.py tests/test_gpu_enumerate.py tests/test_gpu_shard.py tests/test_gpu_w21.py -m gpu -q -x --timeout 300 > gpurun_out/r04u_tests.log 2>&1; rc=$?
grep -E "Error|assert|FAILED|passed|failed" gpurun_out/r04u_tests.log | head -12
exit $rc
