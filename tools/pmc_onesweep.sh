#!/bin/bash
# Wave-cycle breakdown of the onesweep sort passes in the bench (run via gpurun), plus the
# rocPRIM/hipCUB yardstick (development tool).  One rocprofv3 --pmc pass per counter set.
set -o pipefail
OUT=gpurun_out/${1:-pmcq}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NO_YARDSTICK" ]; then
  timeout -k 10 120 ./tools/yardstick_rocprim 800000000 > $OUT/yardstick.txt 2>&1 || exit 10
  cat $OUT/yardstick.txt
fi
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-mums"
RE="onesweep|probe_tile|seed_scatter|seed_pack|ghist"
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $SET --kernel-include-regex "$RE" --output-format csv -d $OUT/p$i -o p -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit $((10+i)); }
done
python3 tools/pmc_summ.py $OUT/p1 $OUT/p2
