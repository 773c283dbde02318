#!/bin/bash
# chain kernel PMC passes (new row layout) + kernel trace of full C3 FindMatches
set -o pipefail
bash tools/pmc_chains.sh r04t_pmc_chains || exit $?
bash tools/prof_c3_mums.sh r04t_c3mums > gpurun_out/r04t_c3mums.txt 2>&1 || { tail -5 gpurun_out/r04t_c3mums.txt; exit 30; }
tail -32 gpurun_out/r04t_c3mums.txt
