#!/bin/bash
# round 5: refilled short-walk lanes (parity, then C3 FindMatches A/B), the seed-scatter
# tile swizzle A/B on the seed stage, then the default bench once (its duration)
set -o pipefail
OUT=gpurun_out/r05l
mkdir -p $OUT
bash tools/gpu_tests.sh r05l tests/test_gpu_walk_refill.py tests/test_gpu_row_paths.py || exit 11
for rep in 1 2; do
  for v in 0 1; do
    MUMS_DEV_WALK_REFILL=$v timeout -k 10 240 python3 -u tools/c3_mums.py 3 > $OUT/refill${v}_r$rep.log 2>&1 \
      || { echo "c3 refill=$v failed"; tail -20 $OUT/refill${v}_r$rep.log; exit 12; }
    echo "refill=$v rep $rep: $(grep '^iter 2' $OUT/refill${v}_r$rep.log)"
  done
done
VAR=MUMS_DEV_LIB VALS="0 libmems_amd/var/libmums_noswz.so" bash tools/ab_env.sh r05l_swz || exit 13
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; tail -20 $OUT/bench.err; exit 14; }
grep '^\[bench' $OUT/bench.err
