#!/bin/bash
# Round 6 first call: per-phase onesweep timing (MUMS_OS_STATS build) + baseline bench of the default library.
set -o pipefail
OUT=gpurun_out/r06a
mkdir -p $OUT
MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_osstats.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-mums --no-cpu-baseline \
  > $OUT/stats.json 2> $OUT/stats.err || { tail -20 $OUT/stats.err; exit 11; }
grep os_stats $OUT/stats.err | tail -8
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 12; }
python3 -c "
import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print(round(d['ms_per_step'],2), 'ms/step onesweep', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],3), d['phase_ms_per_step'], 'mums', d.get('mums_c3',{}).get('ms'))"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_compat.py::test_parallel_c3shape_known_answer" "tests/test_gpu_compat_ranks.py::test_compat_ranks_c3shape_known_answer" \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 13; }
tail -3 $OUT/pytest.log
