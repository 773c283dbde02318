#!/bin/bash
# Segment fix-up timing experiments (MUMS_DEV_SEGFIX=3: no in-place writes, 4: no segment
# sorting; both give wrong results, timing only) vs the default and the onesweep pass.
set -o pipefail
OUT=gpurun_out/${1:-segexp}
mkdir -p $OUT
for V in 1 3 4 0; do
  MUMS_DEV_SEGFIX=$V timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-mums --no-cpu-baseline > $OUT/b$V.json 2> $OUT/b$V.err || { echo "bench failed $V"; tail -5 $OUT/b$V.err; exit 13; }
  python3 -c "
import json; d=json.load(open('$OUT/b$V.json'))
print('segfix=$V', round(d['ms_per_step'],2), 'ms/step', d['phase_ms_per_step'])"
done
