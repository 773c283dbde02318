#!/bin/bash
# round 5: two-pass compat MergeTable (parity incl. the exact pass everywhere), then compat
# FindMatches scaling up to BASELINE config 3
set -o pipefail
OUT=gpurun_out/r05o
mkdir -p $OUT
bash tools/gpu_tests.sh r05o tests/test_gpu_compat.py tests/test_gpu_compat_logs.py tests/test_gpu_tie_order.py tests/test_gpu_walk_refill.py tests/test_gpu_many_genomes.py tests/test_gpu_find_chunked.py || exit 11
timeout -k 10 400 python3 -u tools/dev/compat_scale.py 8 3 10 100 > $OUT/compat_scale.log 2>&1 || { echo "compat scale failed $?"; cat $OUT/compat_scale.log; exit 12; }
cat $OUT/compat_scale.log
