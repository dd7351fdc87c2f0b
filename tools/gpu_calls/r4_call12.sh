bash tools/gpu_steps_safe.sh \
 "r4_pipe_a0:200:python bench.py --steps 20 --warmup 5" \
 "r4_pipe_b0:200:MI355X_DP_KERNEL_VARIANT=pipe python bench.py --steps 20 --warmup 5" \
 "r4_pipe_a1:200:python bench.py --steps 20 --warmup 5" \
 "r4_pipe_b1:200:MI355X_DP_KERNEL_VARIANT=pipe python bench.py --steps 20 --warmup 5" \
 "r4_epi_a:300:python tools/bench_conv_epilogues.py --rounds 2" \
 "r4_epi_b:300:MI355X_DP_KERNEL_VARIANT=pipe python tools/bench_conv_epilogues.py --rounds 2"
