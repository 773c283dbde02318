#!/bin/bash
# A/B seed-stage timing of library variants in one GPU call:  tools/ab.sh tag lib1 lib2 ...
# ("default" = libmems_amd/libmums_hip.so).  Each variant: 2 bench runs, alternating.
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = default ]; then unset MUMS_DEV_LIB; else export MUMS_DEV_LIB=$PWD/$L; fi
    timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-mums --no-cpu-baseline > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err || { echo "FAIL $L"; tail -5 gpurun_out/$T/b.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/$T/b.json')); r=d['roofline']
print('$L', round(d['ms_per_step'],2), 'ms/step', 'onesweep', round(r['avg_launch_ms'],3), 'ms frac', round(r['frac'],3), d['phase_ms_per_step'])"
  done
done
