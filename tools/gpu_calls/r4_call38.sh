bash tools/gpu_steps_safe.sh \
 "r4_t38:400:python -u -m pytest -v --timeout 170 --timeout-method thread tests/test_gpu_integration.py tests/test_transformer_gpu.py tests/test_graph_workspaces_gpu.py -k 'gated_buckets or layernorm or vit or workspace'" &&
bash tools/gpu_steps_safe.sh \
 "r4_l38_vit:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_l38_vit0:300:MI355X_DP_LN_BWD16=0 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_l38_vit1:300:python bench.py --model vit_b_16 --steps 10 --warmup 3"
