bash tools/gpu_steps_safe.sh \
 "r4_t19:400:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_stem_gpu.py tests/test_kernels_gpu.py -k 'stem or entropy or linear or resnet50_bs256'" \
 "r4_bench_nol:300:python tools/bench_nol.py"
