#!/bin/bash
# Closing evidence (round 6 final tree): full GPU suite, smoke, then the round evidence (kernel trace, PMC passes, C3 trace, bench)
set -o pipefail
OUT=gpurun_out/r06zz
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 11; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 12; }
tail -1 $OUT/smoke.log
bash tools/round_evidence.sh r06zz_ev || exit $?
