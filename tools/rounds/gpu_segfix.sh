#!/bin/bash
# One GPU call: the whole GPU parity suite (default sort: onesweep on every digit), incl.
# tests/test_gpu_segfix.py (the opt-in segment fix-up against the oracle).
set -o pipefail
T=${1:-segfix}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed $?"; tail -40 $OUT/pytest_gpu.log; exit 11; }
tail -2 $OUT/pytest_gpu.log
