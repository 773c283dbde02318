#!/bin/bash
# round 4: sharded restart planned on the ranks' own SML parts + every restart path (PlanData accessors)
set -o pipefail
T=r04j
mkdir -p gpurun_out/$T

bash tools/gpu_tests.sh $T tests/test_gpu_shard_restart.py tests/test_gpu_chunked_restart.py tests/test_gpu_restart.py tests/test_gpu_compat.py tests/test_gpu_tie_order.py tests/test_gpu_shard_abi.py -s || exit $?
grep "restart paths" gpurun_out/$T/pytest.log
