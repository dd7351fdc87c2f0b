bash tools/gpu_steps_safe.sh \
 "r4_t49:400:python -u -m pytest tests/test_resblock_gpu.py tests/test_kernels_gpu.py -x -v --timeout 170 --timeout-method thread -k 'block or bits or resnet'" &&
bash tools/gpu_steps_safe.sh \
 "r4_b49:300:python bench.py --steps 20 --warmup 5"
