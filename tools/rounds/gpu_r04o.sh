#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04o
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r04o/bench.json 2> gpurun_out/r04o/bench.err || { tail -20 gpurun_out/r04o/bench.err; exit 3; }
python3 -c "import json; d=json.load(open('gpurun_out/r04o/bench.json')); print(d['ms_per_step'], d['e2e_c3'], d['mums_c3']['ms'])"
