#!/bin/bash
# line hash sort: run-aware histogram + late publish vs plain (MUMS_DEV_LINE_NORUNS), same box
set -o pipefail
for rep in 1 2 3; do
  echo "runs:   $(timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" || exit 1
  echo "noruns: $(MUMS_DEV_LINE_NORUNS=1 timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" || exit 1
done
