#!/bin/bash
# A/B of full C3 FindMatches (chains / replay phases) across library variants in one GPU call:
#   tools/ab_c3mums.sh lib1 lib2 ...   ("default" = libmems_amd/libmums_hip.so)
set -o pipefail
for rep in 1 2; do
  for L in "$@"; do
    if [ "$L" = default ]; then unset MUMS_DEV_LIB; else export MUMS_DEV_LIB=$PWD/$L; fi
    echo "$L: $(timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" || exit 1
  done
done
