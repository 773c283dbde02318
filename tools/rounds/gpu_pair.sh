#!/bin/bash
# paired 16-B onesweep variant: parity (parity shapes + C3 known answer) through MUMS_DEV_LIB, then A/B timing
set -o pipefail
T=${1:-pair}
OUT=gpurun_out/$T
mkdir -p $OUT
MUMS_DEV_LIB=$PWD/libmems_amd/var/libmums_pair.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_gpu_large.py -k "oracle_parity or known_answer or seed_keys or c3" -m gpu -q -x -rf --timeout 200 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 11; }
tail -1 $OUT/pytest.log
bash tools/ab.sh ${T}_ab default libmems_amd/var/libmums_pair.so
