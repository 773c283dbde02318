#!/bin/bash
# One GPU call: a parity subset (parity shapes, sweep, C3 known answer, chunked FindMatches)
# then C3 FindMatches timings.  tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=${2:-}
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_large.py \
  tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py ${K:+-k "$K"} -m gpu -v -x --timeout 200 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 11; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -u tools/c3_mums.py 3 2>&1 | grep iter
