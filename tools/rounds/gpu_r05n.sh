#!/bin/bash
# round 5: ParallelMemHash LogProgress / SetMatchLog parity, then kernel traces of C3
# FindMatches with and without the walk-order sort and of the compat replay (8 x 3 Mbp)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05n
mkdir -p $OUT
bash tools/gpu_tests.sh r05n tests/test_gpu_compat_logs.py tests/test_gpu_progress.py tests/test_gpu_match_log.py tests/test_gpu_compat.py tests/test_gpu_tie_order.py || exit 11
for v in 0 1; do
  MUMS_DEV_WALK_SORT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ws$v -o kt -- python3 -u tools/c3_mums.py 2 > $OUT/ws$v.log 2>&1 || { echo "trace ws$v failed"; tail -20 $OUT/ws$v.log; exit 12; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/compat -o kt -- python3 -u tools/dev/compat_scale.py 8 3 > $OUT/compat.log 2>&1 || { echo "trace compat failed"; tail -20 $OUT/compat.log; exit 13; }
python3 - <<'PY'
import csv, glob
for d in ("ws0", "ws1", "compat"):
    f = glob.glob(f"gpurun_out/r05n/{d}/**/kt_kernel_stats.csv", recursive=True)
    print("==", d, f)
    if not f:
        continue
    for x in list(csv.DictReader(open(f[0])))[:22]:
        print(f"{float(x['TotalDurationNs'])/1e6:9.3f} ms {int(x['Calls']):6d} calls avg {float(x['AverageNs'])/1e3:9.1f} us  {x['Name'][:90]}")
PY
