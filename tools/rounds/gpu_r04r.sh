#!/bin/bash
# int32 line rows for the chain kernels: C3 A/B (64-bit rows via MUMS_DEV_WIDE_LINE_ROWS) + parity
set -o pipefail
for rep in 1 2; do
  echo "narrow: $(timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" || exit 1
  echo "wide:   $(MUMS_DEV_WIDE_LINE_ROWS=1 timeout -k 10 120 python -u tools/c3_mums.py 2 2>/dev/null | tail -1)" || exit 1
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_find_chunked.py tests/test_gpu_many_genomes.py -m gpu -q -x --timeout 200 2>&1 | grep -E "Error|assert|FAILED|passed|failed" | head -8
