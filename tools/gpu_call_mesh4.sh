# IPC mesh collectives with 4 ranks sharing the GPU (one HW queue each: 4 x 4 queues over-subscribe)
export PYTHONPATH=$PWD MI355X_DP_SMDDP_IPC_ONLY=1 MI355X_DP_SMDDP_DEVICE=0 MI355X_DP_SMDDP_IPC_MB=1 GPU_MAX_HW_QUEUES=1
bash tools/gpu_steps.sh \
  mesh2 120 "python -m mi355x_dp.launch --nproc 2 tools/ipc_mesh_check.py" \
  mesh4 150 "python -m mi355x_dp.launch --nproc 4 tools/ipc_mesh_check.py"
