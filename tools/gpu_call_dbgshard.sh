export PYTHONPATH=$PWD MI355X_DP_SMDDP_IPC_ONLY=1 MI355X_DP_SMDDP_DEVICE=0 MI355X_DP_SMDDP_IPC_MB=1
bash tools/gpu_steps.sh \
  dbg2 150 "python -m mi355x_dp.launch --nproc 2 tools/debug_shard2.py" \
  dbg2_ws0 150 "MI355X_DP_WGRAD_STREAM=0 python -m mi355x_dp.launch --nproc 2 tools/debug_shard2.py"
