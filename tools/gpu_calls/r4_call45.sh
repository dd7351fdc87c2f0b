V="python bench.py --model vit_b_16 --steps 10 --warmup 3"
bash tools/gpu_steps_safe.sh \
 "r4_tnv_base:300:$V" \
 "r4_tnv_st2:300:MI355X_DP_TN_STAGES=2 $V" \
 "r4_tnv_b512:300:MI355X_DP_TN_BLOCKS=512 $V" \
 "r4_tnv_b1024:300:MI355X_DP_TN_BLOCKS=1024 $V" \
 "r4_tnv_b1536:300:MI355X_DP_TN_BLOCKS=1536 $V" \
 "r4_tnv_st2b1024:300:MI355X_DP_TN_STAGES=2 MI355X_DP_TN_BLOCKS=1024 $V" \
 "r4_tnv_base1:300:$V"
