bash tools/gpu_steps_safe.sh \
 "r4_gate6_gated:120:python tools/graphed_comm_bench.py --mode gated" \
 "r4_gate6_ungated:120:python tools/graphed_comm_bench.py --mode ungated" \
 "r4_gate6_nccl:120:python tools/graphed_comm_bench.py --mode gated --backend nccl" \
 "r4_gate6_world2:200:MI355X_DP_SMDDP_IPC_ONLY=1 MI355X_DP_SMDDP_DEVICE=0 MI355X_DP_SMDDP_IPC_MB=4 python -m mi355x_dp.launch --nproc 2 tools/graphed_world2.py" \
 "r4_knob_base:200:python bench.py --steps 20 --warmup 5" \
 "r4_knob_tiles256:200:MI355X_DP_CONV256_MIN_TILES=256 python bench.py --steps 20 --warmup 5" \
 "r4_knob_prio:200:MI355X_DP_MAIN_PRIORITY=-1 python bench.py --steps 20 --warmup 5" \
 "r4_knob_tnside256:200:MI355X_DP_TN_BLOCKS_SIDE=256 python bench.py --steps 20 --warmup 5" \
 "r4_knob_tnside512:200:MI355X_DP_TN_BLOCKS_SIDE=512 python bench.py --steps 20 --warmup 5" \
 "r4_knob_base2:200:python bench.py --steps 20 --warmup 5"
