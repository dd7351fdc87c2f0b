bash tools/gpu_steps_safe.sh \
 "r4_g_eager:200:python bench.py --steps 20 --warmup 5" \
 "r4_g_single:300:python bench.py --steps 20 --warmup 5 --graph" \
 "r4_g_multi:300:MI355X_DP_GRAPH_STREAMS=1 python bench.py --steps 20 --warmup 5 --graph" \
 "r4_g_eager1:200:python bench.py --steps 20 --warmup 5" \
 "r4_g_multi1:300:MI355X_DP_GRAPH_STREAMS=1 python bench.py --steps 20 --warmup 5 --graph"
