#!/bin/bash
# Seed-stage A/B on BASELINE config 3 (segment fix-up on / off), then a kernel trace
# of the seed stage with the fix-up.
set -o pipefail
OUT=gpurun_out/${1:-segprof}
mkdir -p $OUT
for rep in 1 2; do
  for V in 1 0; do
    MUMS_DEV_SEGFIX=$V timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-mums --no-cpu-baseline > $OUT/b$V.json 2> $OUT/b$V.err || { echo "bench failed $V"; tail -5 $OUT/b$V.err; exit 13; }
    python3 -c "
import json; d=json.load(open('$OUT/b$V.json')); r=d['roofline']
print('segfix=$V', round(d['ms_per_step'],2), 'ms/step', 'onesweep', round(r['avg_launch_ms'],3), 'ms frac', round(r['frac'],3), d['phase_ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-mums --no-cpu-baseline > $OUT/p.json 2> $OUT/p.err || { tail -5 $OUT/p.err; exit 14; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:12]: print(r['Calls'], round(float(r['AverageNs'])/1e6,3), 'ms', r['Name'][:100])"
