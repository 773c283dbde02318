#!/bin/bash
# One GPU call: the given test files (default: all -m gpu tests), -x, with a per-test limit.
#   tools/gpu_tests.sh <tag> [test paths / -k expressions ...]
set -o pipefail
TAG=${1:-tests}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS=("$@"); [ ${#ARGS[@]} -eq 0 ] && ARGS=(tests)
timeout -k 10 800 python -u -m pytest "${ARGS[@]}" -m gpu -q -x -rf --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 11; }
tail -3 $OUT/pytest.log
