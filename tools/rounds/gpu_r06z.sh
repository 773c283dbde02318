#!/bin/bash
# Pack kernel XCD-grouped tiles A/B (MUMS_DEV_PACK_LINEAR=1: linear tiles) + parity subset +
# per-variant WRITE_SIZE / kernel time of seed_pack_kernel
set -o pipefail
OUT=gpurun_out/${1:-r06z}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_chunked.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 11; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for v in xcd linear; do
    if [ $v = linear ]; then export MUMS_DEV_PACK_LINEAR=1; else unset MUMS_DEV_PACK_LINEAR; fi
    timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-mums > $OUT/b.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 12; }
    python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', round(d['ms_per_step'],3), 'ms/step onesweep', round(r['avg_launch_ms'],3), d['phase_ms_per_step'])"
  done
done
for v in xcd linear; do
  if [ $v = linear ]; then export MUMS_DEV_PACK_LINEAR=1; else unset MUMS_DEV_PACK_LINEAR; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-mums > $OUT/kt_$v.log 2>&1 || exit 13
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_$v -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-mums > $OUT/pmc_$v.log 2>&1 || exit 14
  python3 - <<PY
import csv, glob
rows = list(csv.DictReader(open(glob.glob('$OUT/kt_$v/**/kt_kernel_stats.csv', recursive=True)[0])))
for r in rows:
    if 'seed_pack' in r['Name'] or 'seed_scatter' in r['Name']:
        print('$v', r['Name'][:60], 'calls', r['Calls'], 'avg us', round(float(r['AverageNs'])/1e3, 1))
vals = {}
for f in glob.glob('$OUT/pmc_$v/**/pmc_counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'seed_pack' in r.get('Kernel_Name', ''):
            vals.setdefault(r['Dispatch_Id'], 0.0)
            vals[r['Dispatch_Id']] += float(r['Counter_Value'])
if vals:
    v = sorted(vals.values())
    print('$v seed_pack WRITE_SIZE per dispatch (KiB?):', v[len(v)//2], 'dispatches', len(v))
PY
done
unset MUMS_DEV_PACK_LINEAR
