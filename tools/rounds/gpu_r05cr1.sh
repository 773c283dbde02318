set -o pipefail
mkdir -p gpurun_out/cr1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_compat_ranks.py tests/test_gpu_shard_abi.py::test_shard_run_refuses_single_gpu_modes "tests/test_gpu_cpp_host.py::test_cpp_parallel_compat_known_answer" > gpurun_out/cr1/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/cr1/pytest.log
exit $rc
