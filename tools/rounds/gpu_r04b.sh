#!/bin/bash
# round 4: onesweep claim-ordered descriptors -- parity subset, then A/B against the two-load claim
set -o pipefail
bash tools/gpu_tests.sh r04b tests/test_gpu_parity.py tests/test_gpu_sweep.py tests/test_gpu_w21.py || exit $?
bash tools/ab.sh r04b default libmems_amd/var/libmums_noct.so
