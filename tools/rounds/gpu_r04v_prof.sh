#!/bin/bash
# round-4 final evidence, part 1: chain kernel PMC passes, C3 FindMatches kernel trace, seed-stage profile
set -o pipefail
bash tools/pmc_chains.sh r04v_pmc_chains > gpurun_out/r04v_pmc_chains.txt 2>&1 || { tail -5 gpurun_out/r04v_pmc_chains.txt; exit 21; }
bash tools/prof_c3_mums.sh r04v_c3mums > gpurun_out/r04v_c3mums.txt 2>&1 || { tail -5 gpurun_out/r04v_c3mums.txt; exit 22; }
bash tools/profile_round.sh r04v || exit 23
echo part1 done
