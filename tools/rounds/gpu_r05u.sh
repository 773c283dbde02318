#!/bin/bash
# round 5: short walks binned by genome position (MUMS_DEV_WALK_BINS=1) vs the queue's line
# order: walk parity tests, then kernel traces of C3 FindMatches, two repetitions
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05u
mkdir -p $OUT
bash tools/gpu_tests.sh r05u tests/test_gpu_walk_refill.py tests/test_gpu_row_paths.py tests/test_gpu_parity.py || exit 11
for rep in 1 2; do
  for v in 0 1; do
    MUMS_DEV_WALK_BINS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/wb${v}_$rep -o kt -- python3 -u tools/c3_mums.py 2 > $OUT/wb${v}_$rep.log 2>&1 || { echo "trace wb$v failed"; tail -20 $OUT/wb${v}_$rep.log; exit 12; }
    echo "wb$v rep $rep $(grep '^iter 1' $OUT/wb${v}_$rep.log)"
  done
done
for rep in 1 2; do
  for v in 0 1; do
    MUMS_DEV_WALK_BINS=$v timeout -k 10 200 python3 -u tools/c3_mums.py 4 > $OUT/plain_wb${v}_$rep.log 2>&1 || { echo "plain wb$v failed"; exit 13; }
    echo "plain wb$v rep $rep $(grep '^iter 3' $OUT/plain_wb${v}_$rep.log)"
  done
done
python3 - <<'PY'
import csv
for rep in (1, 2):
    for v in (0, 1):
        rows = list(csv.DictReader(open(f"gpurun_out/r05u/wb{v}_{rep}/kt_kernel_trace.csv")))
        out = []
        for r in rows:
            n = r['Kernel_Name']
            if 'chain_walk' in n or 'walk_bin' in n or 'walk_handoff' in n:
                tag = n.split('(')[0].split('::')[-1].split('<')[0].replace('void ', '')
                out.append((int(r['Start_Timestamp']), tag, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
        out.sort()
        half = out[len(out) // 2:]
        print(f"wb{v} rep{rep}", [(t, round(us)) for _, t, us in half], "sum", round(sum(us for _, _, us in half)))
PY
