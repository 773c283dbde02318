#!/bin/bash
# Same-box A/B of one development switch on the BASELINE config-3 seed stage (bench.py, no
# FindMatches): VAR=<env name> VALS="0 1 ..." (0 = unset), two repetitions, alternating.
#   VAR=MUMS_DEV_OS_XCD VALS="0 1" bash tools/ab_env.sh <tag>
set -o pipefail
TAG=${1:-ab_env}
OUT=gpurun_out/$TAG
mkdir -p $OUT
VAR=${VAR:?set VAR}
VALS=${VALS:-"0 1"}
for rep in 1 2; do
  for v in $VALS; do
    if [ "$v" = 0 ]; then unset $VAR; else export $VAR=$v; fi
    f=$(echo "$v" | tr '/.' '__')
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${EXTRA_ARGS:---no-mums} \
      > $OUT/v${f}_r$rep.json 2> $OUT/v${f}_r$rep.err || { echo "variant $v failed"; tail -20 $OUT/v${f}_r$rep.err; exit 11; }
    python3 - $OUT/v${f}_r$rep.json "$VAR=$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ph = d.get("phase_ms_per_step", {})
r = d.get("roofline", {})
m = d.get("mums_c3", {})
print(f"{sys.argv[2]}: ms/step {d['ms_per_step']:.3f} keys {ph.get('ms_keys')} sort {ph.get('ms_sort')} "
      f"groups {ph.get('ms_groups')} buckets {ph.get('ms_buckets')} | pass {r.get('avg_launch_ms', 0):.3f} ms "
      f"frac {r.get('frac', 0):.3f} | mums {m.get('matches')} {m.get('ms', 0):.1f} ms")
PY
  done
done
