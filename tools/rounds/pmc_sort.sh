#!/bin/bash
# HBM traffic of the onesweep sort passes in tools/sortbench (run via gpurun): FETCH_SIZE and
# WRITE_SIZE in separate passes (MI355X_MICROARCH.md, HBM section).
set -o pipefail
OUT=gpurun_out/pmc_sort_${1:-a}
BIN=${2:-./tools/sortbench_CO}
mkdir -p $OUT
export TMPDIR=/tmp
RE="onesweep|downsweep"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" --output-format csv -d $OUT/f -o f -- $BIN 800000000 7 > $OUT/f.log 2>&1 || exit 11
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RE" --output-format csv -d $OUT/w -o w -- $BIN 800000000 7 > $OUT/w.log 2>&1 || exit 12
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RE" --output-format csv -d $OUT/h -o h -- $BIN 800000000 7 > $OUT/h.log 2>&1 || exit 13
echo done
