#!/bin/bash
# slot occupancy of the default (non-persistent) onesweep pass (stats build)
set -o pipefail
OUT=gpurun_out/r06c
mkdir -p $OUT
MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_osstats.so timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-mums --no-cpu-baseline \
  > $OUT/stats.json 2> $OUT/stats.err || { tail -20 $OUT/stats.err; exit 11; }
grep os_stats $OUT/stats.err | tail -4
