bash tools/gpu_steps_safe.sh \
 "r4_t30:300:python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k layernorm" &&
bash tools/gpu_steps_safe.sh \
 "r4_ln_a:120:MI355X_DP_LN_BWD16=0 python tools/bench_ln.py" \
 "r4_ln_b:120:python tools/bench_ln.py" \
 "r4_vln_a0:300:MI355X_DP_LN_BWD16=0 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_vln_b0:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_vln_a1:300:MI355X_DP_LN_BWD16=0 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_vln_b1:300:python bench.py --model vit_b_16 --steps 10 --warmup 3"
