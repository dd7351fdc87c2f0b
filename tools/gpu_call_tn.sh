bash tools/gpu_steps.sh \
  conv_tests 500 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_resblock_gpu.py tests/test_stem_gpu.py tests/test_gemm256_gpu.py" \
  bench_conv 300 "python tools/bench_conv.py --no-stock" \
  bench 300 "python bench.py --steps 20 --warmup 5"
