#!/bin/bash
# Same-box A/B of the seed-stage sort: four 8-bit onesweep passes (default) against the
# three 10-bit passes of radix_wide.hip (MUMS_DEV_SORT3 = block shape 1/2/3), BASELINE
# config 3, two repetitions each, alternating.  Prints ms_per_step, ms_sort and the
# dominant kernel's HIP-event launch time per variant.
set -o pipefail
TAG=${1:-ab_sort3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
VARS=${VARS:-"0 1 2 3"}
for rep in 1 2; do
  for v in $VARS; do
    if [ "$v" = 0 ]; then unset MUMS_DEV_SORT3; else export MUMS_DEV_SORT3=$v; fi
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${EXTRA_ARGS:---no-mums} \
      > $OUT/v${v}_r$rep.json 2> $OUT/v${v}_r$rep.err || { echo "variant $v failed"; tail -20 $OUT/v${v}_r$rep.err; exit 11; }
    python3 - $OUT/v${v}_r$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ph = d.get("phase_ms_per_step", {})
r = d.get("roofline", {})
m = d.get("mums_c3", {})
print(f"SORT3={sys.argv[2]}: ms/step {d['ms_per_step']:.3f} keys {ph.get('ms_keys')} sort {ph.get('ms_sort')} "
      f"groups {ph.get('ms_groups')} buckets {ph.get('ms_buckets')} | pass {r.get('avg_launch_ms', 0):.3f} ms "
      f"frac {r.get('frac', 0):.3f} | mums {m.get('matches')} {m.get('ms', 0):.1f} ms")
PY
  done
done
