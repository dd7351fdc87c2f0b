V="python bench.py --model vit_b_16 --steps 10 --warmup 3"
bash tools/gpu_steps_safe.sh \
 "r4_aw8:300:$V" \
 "r4_aw4:300:MI355X_DP_ATT_WAVES=4 $V" \
 "r4_aw8b:300:$V" \
 "r4_aw4b:300:MI355X_DP_ATT_WAVES=4 $V"
