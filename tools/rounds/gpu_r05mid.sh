#!/bin/bash
# round 5 mid-session check after the compat-over-ranks, wide walk loads and chain sort changes
set -o pipefail
bash tools/gpu_round.sh r05mid || exit 11
