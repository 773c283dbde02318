#!/bin/bash
# round 5 evidence: boundary / parity / walk-variant tests, the seed-stage profile (kernel
# trace + FETCH/WRITE passes), the C3 FindMatches kernel trace, the bench line, then the
# chain kernels' PMC passes (walk rooflines' counter bytes)
set -o pipefail
bash tools/gpu_tests.sh r05q tests/test_gpu_boundary.py tests/test_gpu_parity.py tests/test_gpu_walk_refill.py tests/test_gpu_cpp_host.py || exit 11
bash tools/round_evidence.sh r05q || exit 12
bash tools/pmc_chains.sh r05q_pmc > /dev/null || exit 13
tail -40 gpurun_out/r05q_pmc/summary.txt
