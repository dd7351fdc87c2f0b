R="python bench.py --model resnet152 --steps 10 --warmup 3"
bash tools/gpu_steps_safe.sh \
 "r4_t152_base:300:$R" \
 "r4_t152_s512:300:MI355X_DP_TN_BLOCKS_SIDE=512 $R" \
 "r4_t152_s640:300:MI355X_DP_TN_BLOCKS_SIDE=640 $R" \
 "r4_t152_b1024:300:MI355X_DP_TN_BLOCKS=1024 $R" \
 "r4_t152_base1:300:$R" \
 "r4_t152_s512b:300:MI355X_DP_TN_BLOCKS_SIDE=512 $R"
