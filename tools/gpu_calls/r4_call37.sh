bash tools/gpu_steps_safe.sh \
 "r4_t37:600:python -u -m pytest -v --timeout 170 --timeout-method thread tests/test_gpu_integration.py tests/test_trajectory_gpu.py tests/test_transformer_gpu.py tests/test_graph_workspaces_gpu.py -k 'gated_buckets or trajectory or layernorm or vit or workspace'" &&
bash tools/gpu_steps_safe.sh \
 "r4_lnf_b0:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_lnf_rn50:200:python bench.py --steps 20 --warmup 5"
