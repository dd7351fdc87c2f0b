timeout -k 10 200 python tools/r18_grad_err.py 2>&1 | grep worst || exit 1
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu > gpurun_out/all_gpu_tests.log 2>&1; tail -5 gpurun_out/all_gpu_tests.log
