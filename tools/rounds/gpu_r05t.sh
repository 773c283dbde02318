#!/bin/bash
# round 5: walk queue orders -- line order (0), position-sorted short walks with the long
# walks sorted back to line order (2) or scattered over the grid (3): kernel traces of C3
# FindMatches, two repetitions
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05t
mkdir -p $OUT
bash tools/gpu_tests.sh r05t tests/test_gpu_walk_refill.py || exit 11
for rep in 1 2; do
  for v in 0 2 3; do
    MUMS_DEV_WALK_SORT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ws${v}_$rep -o kt -- python3 -u tools/c3_mums.py 2 > $OUT/ws${v}_$rep.log 2>&1 || { echo "trace ws$v failed"; tail -20 $OUT/ws${v}_$rep.log; exit 12; }
    echo "ws$v rep $rep $(grep '^iter 1' $OUT/ws${v}_$rep.log)"
  done
done
python3 - <<'PY'
import csv
for rep in (1, 2):
    for v in (0, 2, 3):
        rows = list(csv.DictReader(open(f"gpurun_out/r05t/ws{v}_{rep}/kt_kernel_trace.csv")))
        out = []
        tot = 0.0
        for r in rows:
            n = r['Kernel_Name']
            if 'chain_walk' in n or 'walk_key' in n or 'walk_line_key' in n:
                tag = 'short' if 'short' in n else ('key' if 'walk_key' in n else ('lkey' if 'line_key' in n else ('long16' if ', 16>' in n else 'long64')))
                out.append((int(r['Start_Timestamp']), tag, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
        out.sort()
        half = out[len(out) // 2:]
        print(f"ws{v} rep{rep}", [(t, round(us)) for _, t, us in half], "sum", round(sum(us for _, _, us in half)))
PY
