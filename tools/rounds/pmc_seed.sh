#!/bin/bash
# PMC passes of the seed-stage kernels on BASELINE config 3 (bench.py, 2 steps): HBM
# traffic, wave-cycle split and LDS activity (one rocprofv3 --pmc pass per counter set).
set -o pipefail
OUT=gpurun_out/${1:-pmc_seed}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-mums"
RE="probe_tile_rec|seg_onesweep|seed_scatter|seg_ghist|probe_compact"
i=0
for SET in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $SET --kernel-include-regex "$RE" --output-format csv -d $OUT/p$i -o p -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit $((10+i)); }
done
python3 tools/pmc_summ.py $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 | tee $OUT/summary.txt
