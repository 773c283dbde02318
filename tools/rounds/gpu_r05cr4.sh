set -o pipefail
mkdir -p gpurun_out/cr4
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_shard.py::test_sharded_abi_multiprocess_gpu" > gpurun_out/cr4/pytest.log 2>&1
rc=$?
tail -15 gpurun_out/cr4/pytest.log
exit $rc
