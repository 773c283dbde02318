#!/bin/bash
set -o pipefail
OUT=gpurun_out/r06j
mkdir -p $OUT
MUMS_DEV_SHARD_DEBUG=1 timeout -k 10 400 python3 -u tools/dev/shard_exchange_c3.py 2 50000000 > $OUT/dbg2.txt 2>&1 || { tail -20 $OUT/dbg2.txt; exit 12; }
cat $OUT/dbg2.txt
