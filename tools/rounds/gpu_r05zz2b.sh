#!/bin/bash
# round 5 closing evidence (final code), part 2: the seed-stage profile, the C3 FindMatches trace and a bench line
# (tools/round_evidence.sh), then the chain kernels PMC passes
set -o pipefail
bash tools/round_evidence.sh r05zz2_ev > /dev/null || exit 12
bash tools/pmc_chains.sh r05zz2_pmc > /dev/null || exit 13
echo part2 done
