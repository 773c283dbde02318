#!/bin/bash
# probe-stage VALU cut (record MG left out of the genome lookup): parity, bench; then the
# config-5 restart timing split (tie workspace first try / FindMatches buffers freed)
set -o pipefail
T=${1:-r03q}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_w21.py tests/test_gpu_chunked.py tests/test_gpu_many_genomes.py \
  tests/test_gpu_sweep.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 11; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-mums > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || { tail -20 $OUT/bench_$rep.err; exit 12; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$rep.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3), d['phase_ms_per_step'], round(d['roofline']['frac'],4))"
done
bash tools/gpu_c5tie.sh ${T}_c5 || exit 13
