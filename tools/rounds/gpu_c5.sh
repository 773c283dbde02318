#!/bin/bash
# BASELINE config 5 on one GPU: the reference's default seed for 3 Gbp genomes (w21) and
# N-gapped assemblies (MER_REPEAT_LIMIT restarts in the chunked mode), next to the w19 run.
set -o pipefail
T=${1:-c5}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 400 python -u tools/bench_c5.py --weight 21 --gaps 100 --steps 2 --find-steps 1 > $OUT/w21_gaps.log 2>&1 || { tail -20 $OUT/w21_gaps.log; exit 11; }
tail -1 $OUT/w21_gaps.log
timeout -k 10 400 python -u tools/bench_c5.py --weight 19 --gaps 100 --steps 2 --find-steps 1 > $OUT/w19_gaps.log 2>&1 || { tail -20 $OUT/w19_gaps.log; exit 12; }
tail -1 $OUT/w19_gaps.log
timeout -k 10 400 python -u tools/bench_c5.py --weight 21 --steps 2 --find-steps 1 > $OUT/w21.log 2>&1 || { tail -20 $OUT/w21.log; exit 13; }
tail -1 $OUT/w21.log
