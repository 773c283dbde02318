#!/bin/bash
# round 4: compat truncation, tie order, progress, chunked restart parity; then a short bench
set -o pipefail
bash tools/gpu_tests.sh r04a tests/test_gpu_compat.py tests/test_gpu_tie_order.py tests/test_gpu_progress.py \
  tests/test_gpu_chunked_restart.py || exit $?
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err \
  || { echo bench failed; tail -20 gpurun_out/r04a/bench.err; exit 12; }
tail -c 3000 gpurun_out/r04a/bench.json
