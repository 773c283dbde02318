#!/bin/bash
# HBM traffic and wave-cycle split of the FindMatches chain kernels on BASELINE config 3
# (run via gpurun): one rocprofv3 --pmc pass per counter set (FETCH_SIZE x 2 on gfx950 for
# wide streaming reads, MI355X_MICROARCH.md), then the per-dispatch summary.
set -o pipefail
OUT=gpurun_out/${1:-pmc_chains}
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 tools/c3_mums.py 1"
RE="chain_|replay|bigg_|bigq_|gather_rows|probe_materialize|keep_fill|kept_summary"
i=0
for SET in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD" \
           "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $SET --kernel-include-regex "$RE" --output-format csv -d $OUT/p$i -o p -- $CMD > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit $((10+i)); }
done
python3 tools/pmc_summ.py $OUT/p1 $OUT/p2 $OUT/p3 $OUT/p4 | tee $OUT/summary.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $CMD > $OUT/kt.log 2>&1 || exit 20
python3 - <<PY
import csv
r = list(csv.DictReader(open("$OUT/kt/kt_kernel_stats.csv")))
with open("$OUT/kernel_stats.txt", "w") as f:
    for x in r[:20]:
        f.write(f"{float(x['AverageNs'])/1e3:10.1f} us avg {int(x['Calls']):4d} calls {float(x['TotalDurationNs'])/1e6:9.3f} ms total  {x['Name'][:110]}\n")
print(open("$OUT/kernel_stats.txt").read())
PY
