#!/bin/bash
# Short-walk queue order A/B at C3 FindMatches: line order (default), position order with the
# 2^11-column granule (MUMS_DEV_WALK_SORT=2, 16 key bits = 2 sort passes), and a coarse one-pass
# granule (MUMS_DEV_WALK_SHIFT=19: 8 key bits at 100 Mbp genomes)
set -o pipefail
OUT=gpurun_out/${1:-r06w2}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_walk_refill.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 11; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for v in line pos16 pos8; do
    unset MUMS_DEV_WALK_SORT MUMS_DEV_WALK_SHIFT
    if [ $v = pos16 ]; then export MUMS_DEV_WALK_SORT=2; fi
    if [ $v = pos8 ]; then export MUMS_DEV_WALK_SORT=2; export MUMS_DEV_WALK_SHIFT=19; fi
    timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-compat > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 12; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); m=d['mums_c3']
print('$v', 'C3 FindMatches', round(m['ms'],2), 'ms', m['phase_ms'], 'matches', m['matches'])"
  done
done
