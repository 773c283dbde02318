#!/bin/bash
# SQ counters for a development kernel binary (run via gpurun): $1 tag, $2 binary, $3.. args
set -o pipefail
OUT=gpurun_out/pmc_local_$1
BIN=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/a -o a -- $BIN "$@" > $OUT/a.log 2>&1 || exit 11
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o b -- $BIN "$@" > $OUT/b.log 2>&1 || exit 12
echo done
