# stream knobs re-checked now that every stream has its own hardware queue (GPU_MAX_HW_QUEUES=8)
B="python bench.py --steps 30 --warmup 5"
bash tools/gpu_steps.sh \
  k8_base 120 "$B" \
  k8_ds 120 "MI355X_DP_DS_STREAM=1 $B" \
  k8_prio 120 "MI355X_DP_WGRAD_PRIORITY=-1 $B" \
  k8_tn256 120 "MI355X_DP_TN_BLOCKS_SIDE=256 $B" \
  k8_tn512 120 "MI355X_DP_TN_BLOCKS_SIDE=512 $B" \
  k8_base2 120 "$B" \
  k8_ds2 120 "MI355X_DP_DS_STREAM=1 $B" \
  k8_prio2 120 "MI355X_DP_WGRAD_PRIORITY=-1 $B" \
  k8_q4 120 "MI355X_DP_HW_QUEUES=0 $B" \
  k8_q16 120 "MI355X_DP_HW_QUEUES=16 $B"
