#!/bin/bash
# round 5 closing evidence (final code), part 1: the whole -m gpu suite, smoke and the bench
set -o pipefail
bash tools/gpu_round.sh r05zz2 || exit 11
echo part1 done
