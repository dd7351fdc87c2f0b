bash tools/gpu_steps_safe.sh \
 "r4_tns_a0:200:python bench.py --steps 20 --warmup 5" \
 "r4_tns_b0:200:MI355X_DP_TN_STAGES=2 python bench.py --steps 20 --warmup 5" \
 "r4_tns_a1:200:python bench.py --steps 20 --warmup 5" \
 "r4_tns_b1:200:MI355X_DP_TN_STAGES=2 python bench.py --steps 20 --warmup 5" \
 "r4_tns_c0:200:MI355X_DP_TN_STAGES=2 MI355X_DP_TN_BLOCKS_SIDE=256 python bench.py --steps 20 --warmup 5" \
 "r4_tns_vit_b:300:MI355X_DP_TN_STAGES=2 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_tns_vit_a:300:python bench.py --model vit_b_16 --steps 10 --warmup 3"
