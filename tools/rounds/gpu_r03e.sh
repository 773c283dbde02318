#!/bin/bash
set -o pipefail
T=${1:-r03e}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_w21.py tests/test_gpu_parity.py tests/test_gpu_chunked.py \
  tests/test_gpu_chunked_restart.py -m gpu -v -x -rf --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 \
  || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 11; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u tools/seed_patterns_bench.py --patterns 21:0,19:0 --tag split > $OUT/pat.jsonl 2> $OUT/pat.err || { tail -5 $OUT/pat.err; exit 12; }
cat $OUT/pat.jsonl
bash tools/gpu_c5.sh ${T}_c5
