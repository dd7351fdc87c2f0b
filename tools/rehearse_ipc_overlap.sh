#!/bin/bash
# Two bench.py ranks on ONE GPU over the native smddp backend in IPC-only mode (no RCCL: RCCL
# refuses two ranks per device), each under its own rocprofv3 --kernel-trace: the per-rank traces
# show the IPC all-reduce kernels of every gradient bucket on the comm stream interleaved with the
# backward kernels on the compute stream.  Outputs: gpurun_out/ipc_overlap_r{0,1}/, *.log
#   bash tools/rehearse_ipc_overlap.sh [MODEL] [BATCH] [STEPS]
MODEL=${1:-resnet50}; BATCH=${2:-64}; STEPS=${3:-6}
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 WORLD_SIZE=2 MI355X_DP_SMDDP_IPC_ONLY=1
export MI355X_DP_SMDDP_DEVICE=0 MI355X_DP_SMDDP_IPC_MB=32 MI355X_DP_SMDDP_TERMINATE_TRACE=1
mkdir -p gpurun_out
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ipc_overlap_r$r -o run -- \
    python3 bench.py --gpus 2 --backend smddp --model $MODEL --batch $BATCH --steps $STEPS --warmup 2 \
    > gpurun_out/ipc_overlap_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
grep '^{' gpurun_out/ipc_overlap_r0.log
exit $rc
