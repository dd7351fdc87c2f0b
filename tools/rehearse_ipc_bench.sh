#!/bin/bash
# Two bench.py ranks on ONE GPU over the native smddp backend in IPC-only mode (no RCCL).
#   bash tools/rehearse_ipc_bench.sh [MODEL] [BATCH] [STEPS] [extra bench args...]
MODEL=${1:-resnet50}; BATCH=${2:-64}; STEPS=${3:-6}; shift 3
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29562 WORLD_SIZE=2 MI355X_DP_SMDDP_IPC_ONLY=1
export MI355X_DP_SMDDP_DEVICE=0 MI355X_DP_SMDDP_IPC_MB=${MI355X_DP_SMDDP_IPC_MB:-32} MI355X_DP_SMDDP_TERMINATE_TRACE=1
export MI355X_DP_BENCH_STACKS=${MI355X_DP_BENCH_STACKS:-50}
mkdir -p gpurun_out
pids=()
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 200 python3 -u bench.py --gpus 2 --backend smddp --model $MODEL --batch $BATCH \
    --steps $STEPS --warmup 2 "$@" > gpurun_out/ipc_bench_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
grep '^{' gpurun_out/ipc_bench_r0.log
exit $rc
