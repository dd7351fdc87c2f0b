bash tools/gpu_steps_safe.sh \
 "r4_t31:300:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k 'vit or layernorm'" &&
bash tools/gpu_steps_safe.sh \
 "r4_vemb_a0:300:MI355X_DP_VIT_EMBED=0 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_vemb_b0:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_vemb_a1:300:MI355X_DP_VIT_EMBED=0 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_vemb_b1:300:python bench.py --model vit_b_16 --steps 10 --warmup 3"
