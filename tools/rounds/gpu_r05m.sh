#!/bin/bash
# round 5: walk queue in genome-position order (C3 FindMatches A/B), the compat FindMatches
# scaling probe, then the whole -m gpu suite with the new defaults
set -o pipefail
OUT=gpurun_out/r05m
mkdir -p $OUT
for rep in 1 2; do
  for v in 0 1; do
    MUMS_DEV_WALK_SORT=$v timeout -k 10 240 python3 -u tools/c3_mums.py 3 > $OUT/wsort${v}_r$rep.log 2>&1 \
      || { echo "c3 wsort=$v failed"; tail -20 $OUT/wsort${v}_r$rep.log; exit 12; }
    echo "wsort=$v rep $rep: $(grep '^iter 2' $OUT/wsort${v}_r$rep.log)"
  done
done
timeout -k 10 300 python3 -u tools/dev/compat_scale.py 8 1 3 10 > $OUT/compat_scale.log 2>&1 || { echo "compat scale failed $?"; tail -20 $OUT/compat_scale.log; }
cat $OUT/compat_scale.log
bash tools/gpu_tests.sh r05m || exit 11
