#!/bin/bash
# round 5: parity of the sharded enumeration / chain labelling / XCD queues / LDS genome lookup,
# then same-box A/Bs of the XCD claim queues and the genome lookup (seed stage, C3)
set -o pipefail
bash tools/gpu_tests.sh r05j tests/test_gpu_shard_abi.py tests/test_gpu_shard_restart.py tests/test_gpu_sort3.py tests/test_gpu_parity.py -k "shard_chains or bucket_owner or refuses or gathered or undecidable or enumeration or xcd or parity" || exit 11
VAR=MUMS_DEV_OS_XCD VALS="0 1" bash tools/ab_env.sh r05j_xcd || exit 12
VAR=MUMS_DEV_NO_GL VALS="0 1" bash tools/ab_env.sh r05j_gl || exit 13
