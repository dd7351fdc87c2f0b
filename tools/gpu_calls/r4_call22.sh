bash tools/gpu_steps_safe.sh \
 "r4_t22:500:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resblock_gpu.py tests/test_kernels_gpu.py -k 'fused or resnet50_bs256 or resnet18_train or normalize or mask_bits'" &&
bash tools/gpu_steps_safe.sh \
 "r4_ibits_a0:200:MI355X_DP_INNER_BITS=0 python bench.py --steps 20 --warmup 5" \
 "r4_ibits_b0:200:python bench.py --steps 20 --warmup 5" \
 "r4_ibits_a1:200:MI355X_DP_INNER_BITS=0 python bench.py --steps 20 --warmup 5" \
 "r4_ibits_b1:200:python bench.py --steps 20 --warmup 5"
