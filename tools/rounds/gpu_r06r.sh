#!/bin/bash
# Direct compat records with the parallel block digits / in-block screen: parity + C3 A/B + kernel trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06r}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_compat.py tests/test_gpu_compat_logs.py tests/test_gpu_tie_order.py tests/test_gpu_compat_ranks.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py tests/test_gpu_chunked.py tests/test_gpu_restart.py tests/test_gpu_shard_restart.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 12; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
  MUMS_DEV_COMPAT_DEBUG=1 timeout -k 10 300 python3 -u tools/dev/compat_c3.py 3 > $OUT/c3_direct.log 2>&1 || { tail -20 $OUT/c3_direct.log; exit 13; }
  grep -a "iter\|compat direct" $OUT/c3_direct.log | tail -2
  MUMS_DEV_COMPAT_PART=1 timeout -k 10 300 python3 -u tools/dev/compat_c3.py 3 > $OUT/c3_part.log 2>&1 || { tail -20 $OUT/c3_part.log; exit 14; }
  grep -a "iter" $OUT/c3_part.log | tail -1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 -u tools/dev/compat_c3.py 3 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 15; }
python3 - <<PY
import csv
r = list(csv.DictReader(open("$OUT/kt/kt_kernel_stats.csv")))
for x in r:
    n = x['Name']
    if any(k in n for k in ("cd_", "cr_", "compat_", "seg_onesweep_kernel<768, 12, true, false, false>", "seg_ghist", "scan_")):
        print(f"{float(x['TotalDurationNs'])/1e6/3:9.3f} ms/iter {int(x['Calls'])/3:6.1f} calls avg {float(x['AverageNs'])/1e3:9.1f} us  {n[:100]}")
PY
