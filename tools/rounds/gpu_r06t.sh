#!/bin/bash
# Compat chunk starts from the sorted stream (no genome-major SMLs): parity + C3 A/B (MUMS_DEV_COMPAT_SML) + trace
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06t}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_compat.py -k "direct or known or c3shape" > $OUT/direct.log 2>&1 || { tail -40 $OUT/direct.log; exit 11; }
grep -a "compat fast\|passed\|failed" $OUT/direct.log | sort | uniq -c | tail -8
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_compat.py tests/test_gpu_compat_logs.py tests/test_gpu_tie_order.py tests/test_gpu_compat_ranks.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py tests/test_gpu_chunked.py tests/test_gpu_restart.py tests/test_gpu_shard_restart.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 12; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
  MUMS_DEV_COMPAT_DEBUG=1 timeout -k 10 300 python3 -u tools/dev/compat_c3.py 3 > $OUT/c3_lean.log 2>&1 || { tail -20 $OUT/c3_lean.log; exit 13; }
  grep -a "iter\|compat" $OUT/c3_lean.log | tail -3
  MUMS_DEV_COMPAT_SML=1 timeout -k 10 300 python3 -u tools/dev/compat_c3.py 3 > $OUT/c3_sml.log 2>&1 || { tail -20 $OUT/c3_sml.log; exit 14; }
  grep -a "iter" $OUT/c3_sml.log | tail -1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 -u tools/dev/compat_c3.py 3 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 15; }
python3 - <<PY
import csv
r = list(csv.DictReader(open("$OUT/kt/kt_kernel_stats.csv")))
for x in r:
    n = x['Name']
    if any(k in n for k in ("cd_", "cr_", "compat_", "seg_onesweep_kernel<768, 12, true, false, false>", "seg_ghist")):
        print(f"{float(x['TotalDurationNs'])/1e6/3:9.3f} ms/iter {int(x['Calls'])/3:6.1f} calls avg {float(x['AverageNs'])/1e3:9.1f} us  {n[:100]}")
PY
