#!/bin/bash
# round 5: walk kernels with the XCD-grouped block order (default build) vs without
# (var/libmums_noswz.so), each with the walk queue in line order and position-sorted
# (2: the handed-on long walks sorted back into line order):
# kernel traces of C3 FindMatches
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05p
mkdir -p $OUT
bash tools/gpu_tests.sh r05p tests/test_gpu_walk_refill.py tests/test_gpu_parity.py tests/test_gpu_row_paths.py || exit 11
for lib in swz noswz; do
  for v in 0 1 2; do
    [ $lib = noswz ] && [ $v = 2 ] && continue
    if [ $lib = noswz ]; then export MUMS_DEV_LIB=libmems_amd/var/libmums_noswz.so; else unset MUMS_DEV_LIB; fi
    MUMS_DEV_WALK_SORT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${lib}_ws$v -o kt -- python3 -u tools/c3_mums.py 2 > $OUT/${lib}_ws$v.log 2>&1 || { echo "trace $lib ws$v failed"; tail -20 $OUT/${lib}_ws$v.log; exit 12; }
    grep "^iter 1" $OUT/${lib}_ws$v.log
  done
done
unset MUMS_DEV_LIB
python3 - <<'PY'
import csv
for lib in ("swz", "noswz"):
    for d in ("ws0", "ws1", "ws2"):
        if lib == "noswz" and d == "ws2":
            continue
        rows = list(csv.DictReader(open(f"gpurun_out/r05p/{lib}_{d}/kt_kernel_trace.csv")))
        out = []
        for r in rows:
            n = r['Kernel_Name']
            if 'chain_walk' in n or 'walk_key' in n:
                tag = 'short' if 'short' in n else ('key' if 'walk_key' in n else ('long16' if ', 16>' in n else 'long64'))
                out.append((int(r['Start_Timestamp']), tag, (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
        out.sort()
        print(lib, d, [(t, round(us)) for _, t, us in out[len(out) // 2:]])
PY
