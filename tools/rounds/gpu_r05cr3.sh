set -o pipefail
mkdir -p gpurun_out/cr3
export TMPDIR=/tmp MUMS_DEV_COMPAT_RANK_DEBUG=1
timeout -k 10 400 python -u tools/dev/compat_ranks_c3.py 2 > gpurun_out/cr3/w2.log 2>&1 && \
timeout -k 10 400 python -u tools/dev/compat_ranks_c3.py 4 > gpurun_out/cr3/w4.log 2>&1
rc=$?
cat gpurun_out/cr3/w2.log; cat gpurun_out/cr3/w4.log 2>/dev/null
exit $rc
