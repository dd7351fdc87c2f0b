bash tools/gpu_steps_safe.sh \
 "r4_ts_vit_a:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_ts_vit_b:300:MI355X_DP_TAIL_SPLIT=0 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_ts_vit_c:300:MI355X_DP_TAIL_MIN_KT=6 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_ts_vit_a1:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_ts_vit_b1:300:MI355X_DP_TAIL_SPLIT=0 python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_ts_rn_a:200:python bench.py --steps 20 --warmup 5" \
 "r4_ts_rn_b:200:MI355X_DP_TAIL_SPLIT=0 python bench.py --steps 20 --warmup 5"
