#!/bin/bash
# PMC counters for the seed-stage kernels (run via gpurun). Separate passes per counter group.
set -o pipefail
OUT=gpurun_out/pmc_${1:-a}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-mums"
RE="probe_tile|seed_scatter|seed_pack"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --kernel-include-regex "$RE" --output-format csv -d $OUT/sq -o sq -- $CMD > $OUT/sq.log 2>&1 || exit 11
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RE" --output-format csv -d $OUT/tcc -o tcc -- $CMD > $OUT/tcc.log 2>&1 || exit 12
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-include-regex "$RE" --output-format csv -d $OUT/sq2 -o sq2 -- $CMD > $OUT/sq2.log 2>&1 || exit 13
timeout -k 10 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum --kernel-include-regex "$RE" --output-format csv -d $OUT/ta -o ta -- $CMD > $OUT/ta.log 2>&1 || echo "ta pass failed"
echo done
