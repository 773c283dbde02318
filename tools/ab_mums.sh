#!/bin/bash
# A/B FindMatches timing (BASELINE config-2 shape, related and iid) of library variants in
# one GPU call:   tools/ab_mums.sh lib1 lib2 ...   ("default" = libmems_amd/libmums_hip.so)
set -o pipefail
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = default ]; then unset MUMS_DEV_LIB; else export MUMS_DEV_LIB=$PWD/$L; fi
    echo "== $L"
    timeout -k 10 120 python tools/replay_dbg.py 2>&1 | grep "iter 1" || exit 1
    timeout -k 10 120 python tools/replay_dbg.py 4 10000000 1.0 2>&1 | grep "iter 1" || exit 1
  done
done
