bash tools/gpu_steps_safe.sh \
 "r4_stem_a0:200:python bench.py --steps 20 --warmup 5" \
 "r4_stem_b0:200:MI355X_DP_STEM_BLOCKS=512 python bench.py --steps 20 --warmup 5" \
 "r4_stem_c0:200:MI355X_DP_STEM_BLOCKS=1024 python bench.py --steps 20 --warmup 5" \
 "r4_stem_a1:200:python bench.py --steps 20 --warmup 5" \
 "r4_stem_b1:200:MI355X_DP_STEM_BLOCKS=512 python bench.py --steps 20 --warmup 5" \
 "r4_stem_c1:200:MI355X_DP_STEM_BLOCKS=1024 python bench.py --steps 20 --warmup 5"
