bash tools/gpu_steps_safe.sh \
 "r4_gate5_gated:120:python tools/graphed_comm_bench.py --mode gated" \
 "r4_gate5_ungated:120:python tools/graphed_comm_bench.py --mode ungated" \
 "r4_prof_grid:400:bash tools/r4_prof_grid.sh r4_rn50" \
 "r4_conv_s1:300:python tools/bench_conv.py --no-stock --stages 1" \
 "r4_conv_s2:300:python tools/bench_conv.py --no-stock --stages 2"
