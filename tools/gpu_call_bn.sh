bash tools/gpu_steps.sh \
  bench_bn 200 "python tools/bench_bn.py" \
  bn_tests 300 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'batchnorm or resnet18_train'" \
  bench 300 "python bench.py --steps 20 --warmup 5"
