#!/bin/bash
# Compat C3 kernel trace (where the 20 ms over MemHash's sort goes)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06o}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/dev/compat_c3.py 3 > $OUT/plain.log 2>&1 || { tail -20 $OUT/plain.log; exit 10; }
cat $OUT/plain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 -u tools/dev/compat_c3.py 3 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 11; }
python3 - <<PY
import csv
r = list(csv.DictReader(open("$OUT/kt/kt_kernel_stats.csv")))
for x in r[:45]:
    print(f"{float(x['TotalDurationNs'])/1e6/3:9.3f} ms/iter {int(x['Calls'])/3:6.1f} calls avg {float(x['AverageNs'])/1e3:9.1f} us  {x['Name'][:110]}")
PY
