bash tools/gpu_steps_safe.sh \
 "r4_t34:400:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_transformer_gpu.py -k 'transposed or resnet50_bs256 or linear or vit or gemm'" &&
bash tools/gpu_steps_safe.sh \
 "r4_b34_rn50:200:python bench.py --steps 20 --warmup 5" \
 "r4_b34_vit:300:python bench.py --model vit_b_16 --steps 10 --warmup 3"
