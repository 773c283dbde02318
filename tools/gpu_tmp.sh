set -o pipefail
T=${1:-s2e}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1; rc=$?
tail -25 gpurun_out/$T/pytest.log
[ $rc -eq 0 ] || exit $rc
MUMS_DEV_REPLAY_DEBUG=1 timeout -k 10 200 python tools/replay_dbg.py 2>&1 | tail -8
