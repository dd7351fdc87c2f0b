bash tools/gpu_steps_safe.sh \
 "r4_t44:300:python -u -m pytest -v --timeout 170 --timeout-method thread tests/test_transformer_gpu.py -k 'attention or vit or encoder'" &&
bash tools/gpu_steps_safe.sh \
 "r4_att_a:120:MI355X_DP_ATT_PREFETCH=0 python tools/bench_attention.py" \
 "r4_att_b:120:python tools/bench_attention.py" \
 "r4_apf_vit_a:300:MI355X_DP_ATT_PREFETCH=0 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_apf_vit_b:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_apf_vit_a1:300:MI355X_DP_ATT_PREFETCH=0 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_apf_vit_b1:300:python bench.py --model vit_b_16 --steps 10 --warmup 3"
