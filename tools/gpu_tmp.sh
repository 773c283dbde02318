timeout -k 10 300 python -u -m pytest tests/test_gpu_cpp_host.py -x -q --timeout 200 --timeout-method thread > gpurun_out/cpp.log 2>&1; tail -3 gpurun_out/cpp.log
