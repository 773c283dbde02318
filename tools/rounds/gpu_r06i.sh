#!/bin/bash
set -o pipefail
OUT=gpurun_out/r06i
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/dev/shard_exchange_c3.py 4 > $OUT/shard_exchange_c3_w4.txt 2>&1 || { tail -20 $OUT/shard_exchange_c3_w4.txt; exit 11; }
cat $OUT/shard_exchange_c3_w4.txt
