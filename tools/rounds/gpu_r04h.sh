#!/bin/bash
# round 4: sharded w20-21 above 2^32 (IB33 forced), bucket-sort onesweep A/B, C5 arena FindMatches
set -o pipefail
T=r04h
OUT=gpurun_out/$T
mkdir -p $OUT
bash tools/gpu_tests.sh $T tests/test_gpu_shard_abi.py tests/test_gpu_shard.py tests/test_gpu_parity.py \
  tests/test_gpu_restart.py tests/test_gpu_shard_restart.py || exit $?
for rep in 1 2; do
  for v in os radix; do
    E=""; [ $v = radix ] && E="MUMS_DEV_BUCKET_RADIX=1"
    env $E timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-mums --no-cpu-baseline > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -5 $OUT/b_$v.err; exit 12; }
    python3 -c "import json; d=json.load(open('$OUT/b_$v.json')); print('$v', round(d['ms_per_step'],2), d['phase_ms_per_step'], round(d['roofline']['avg_launch_ms'],3))"
  done
done
MUMS_DEV_RESTART_TIMING=1 timeout -k 10 600 python -u tools/bench_c5.py --weight 21 --gaps 100 --steps 1 --find-steps 3 > $OUT/c5.log 2>&1 || { tail -20 $OUT/c5.log; exit 13; }
grep -E "restart phase tie workspace|FindMatches [0-9]|step " $OUT/c5.log | tail -14
tail -1 $OUT/c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); f=d['findmatches']; print('seed ms/step', d['ms_per_step'], d['phase_ms'], 'find ms', f['ms'], f['matches'], f['phase_ms'])"
