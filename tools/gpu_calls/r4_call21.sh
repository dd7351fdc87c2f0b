bash tools/gpu_steps_safe.sh \
 "r4_t21:500:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_resblock_gpu.py -k 'mask_bits or fused or resnet50_bs256 or resnet18_train or normalize'" &&
bash tools/gpu_steps_safe.sh \
 "r4_bits_a0:200:MI355X_DP_OUT_BITS=0 python bench.py --steps 20 --warmup 5" \
 "r4_bits_b0:200:python bench.py --steps 20 --warmup 5" \
 "r4_bits_a1:200:MI355X_DP_OUT_BITS=0 python bench.py --steps 20 --warmup 5" \
 "r4_bits_b1:200:python bench.py --steps 20 --warmup 5"
