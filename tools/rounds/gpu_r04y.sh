#!/bin/bash
# bucket sort upsweep: per-key LDS atomics (default) vs wave-aggregated digit counts (MUMS_DEV_RS_AGG), same box
set -o pipefail
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-mums"
for rep in 1 2; do
  echo "plain: $(timeout -k 10 200 $B 2>/dev/null | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["phase_ms_per_step"])')" || exit 1
  echo "agg:   $(MUMS_DEV_RS_AGG=1 timeout -k 10 200 $B 2>/dev/null | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["ms_per_step"], d["phase_ms_per_step"])')" || exit 1
done
echo "c3: $(timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)"
MUMS_DEV_RS_AGG=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -q -x --timeout 200 2>&1 | grep -E "passed|failed|Error" | head -5
