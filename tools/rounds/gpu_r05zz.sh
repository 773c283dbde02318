#!/bin/bash
# round 5 closing evidence with the final code: the whole -m gpu suite, smoke and the bench
# (tools/gpu_round.sh), then the seed-stage profile, the C3 FindMatches trace and a bench line
# (tools/round_evidence.sh) and the chain kernels' PMC passes
set -o pipefail
bash tools/gpu_round.sh r05zz || exit 11
bash tools/round_evidence.sh r05zz_ev > /dev/null || exit 12
bash tools/pmc_chains.sh r05zz_pmc > /dev/null || exit 13
echo evidence done
