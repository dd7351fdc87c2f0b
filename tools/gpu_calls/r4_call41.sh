bash tools/gpu_steps_safe.sh \
 "r4_t41:400:python -u -m pytest -v --timeout 170 --timeout-method thread tests/test_gpu_integration.py tests/test_kernels_gpu.py tests/test_stem_gpu.py tests/test_transformer_gpu.py -k 'gated_buckets or resnet50_bs256 or batchnorm or bn_ or stem or vit or resblock'" &&
bash tools/gpu_steps_safe.sh \
 "r4_prof41:400:bash tools/r4_prof_grid.sh r4_p41" \
 "r4_b41_a:200:python bench.py --steps 20 --warmup 5" \
 "r4_b41_b:200:python bench.py --steps 20 --warmup 5"
