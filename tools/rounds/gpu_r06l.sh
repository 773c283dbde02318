#!/bin/bash
# Lean walk kernels (no generic hit-word path; 4 waves/SIMD) A/B on C3 FindMatches + chain parity
set -o pipefail
OUT=gpurun_out/r06l
mkdir -p $OUT
for rep in 1 2; do
  for v in gen lean wpe0; do
    unset MUMS_DEV_LIB MUMS_DEV_WALK_GEN
    [ $v = gen ] && export MUMS_DEV_WALK_GEN=1
    [ $v = wpe0 ] && export MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_wpe0.so
    timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-compat > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 12; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); m=d['mums_c3']
print('$v', round(d['ms_per_step'],2), 'ms/step | C3 FindMatches', round(m['ms'],2), 'ms chains', m['phase_ms']['ms_chains'], 'short', round(m['roofline']['ms'],3), 'long', round(m['roofline_long_walks']['ms'],3), m.get('matches'))"
  done
done
unset MUMS_DEV_LIB MUMS_DEV_WALK_GEN
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_walk_refill.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 13; }
tail -2 $OUT/pytest.log
