#!/bin/bash
# 4 gloo ranks sharing one GPU, ResNet-50 bs64, default bucket plan (round-1 stall rehearsal).
#   bash tools/rehearse_gloo4.sh [extra bench args]
export MI355X_DP_BENCH_STACKS=${MI355X_DP_BENCH_STACKS:-40}
timeout -k 10 170 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29571 bench.py --gpus 4 --backend gloo --model resnet50 --batch 64 --steps 3 --warmup 1 "$@"
