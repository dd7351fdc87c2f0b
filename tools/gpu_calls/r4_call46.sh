R="python bench.py --steps 20 --warmup 5"
bash tools/gpu_steps_safe.sh \
 "r4_tnr_base:300:$R" \
 "r4_tnr_s256:300:MI355X_DP_TN_BLOCKS_SIDE=256 $R" \
 "r4_tnr_s320:300:MI355X_DP_TN_BLOCKS_SIDE=320 $R" \
 "r4_tnr_s448:300:MI355X_DP_TN_BLOCKS_SIDE=448 $R" \
 "r4_tnr_s512:300:MI355X_DP_TN_BLOCKS_SIDE=512 $R" \
 "r4_tnr_base1:300:$R" \
 "r4_tnr_s448b:300:MI355X_DP_TN_BLOCKS_SIDE=448 $R" \
 "r4_tnr_s320b:300:MI355X_DP_TN_BLOCKS_SIDE=320 $R"
