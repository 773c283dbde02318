#!/bin/bash
# round 4: sharded restart planned on the ranks' own SML parts + every restart path (PlanData accessors)
set -o pipefail
T=r04j
mkdir -p gpurun_out/$T
MUMS_DEV_SHARD_RESTART_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_restart.py -m gpu -q -x -k "n_gapped and blocks-2" > gpurun_out/$T/dbg.log 2>&1; grep -E "^rank|Error|error|passed|failed" gpurun_out/$T/dbg.log | head -40
bash tools/gpu_tests.sh $T tests/test_gpu_shard_restart.py tests/test_gpu_chunked_restart.py tests/test_gpu_restart.py tests/test_gpu_compat.py tests/test_gpu_tie_order.py tests/test_gpu_shard_abi.py -s || exit $?
grep "restart paths" gpurun_out/$T/pytest.log
