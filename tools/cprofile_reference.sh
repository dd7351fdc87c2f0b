#!/bin/bash
# cProfile of the UNMODIFIED reference GPU script (1 epoch) with the job env; top host functions
#   bash tools/cprofile_reference.sh [BATCH] [ENGINE_DDP 1|0]
set -e
BATCH=${1:-32}
ENGINE=${2:-1}
REPO=$(pwd)
mkdir -p gpurun_out /tmp/cpmodel
python -c "import sys; sys.path.insert(0, '$REPO'); from mi355x_dp.data.cifar import write_synthetic_cifar10 as w; w('/tmp/cpcifar')"
export SM_HOSTS='["algo-1"]' SM_CURRENT_HOST=algo-1 SM_MODEL_DIR=/tmp/cpmodel SM_CHANNEL_TRAIN=/tmp/cpcifar
export LOCAL_RANK=0 RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29519
export PYTHONPATH=$REPO:$REPO/compat MI355X_DP_ENGINE_DDP=$ENGINE
SCRIPT=ref_fixture/notebooks/code/cifar10-distributed-smddp-gpu.py
timeout -k 10 300 python -m cProfile -o /tmp/ref.prof $SCRIPT --backend smddp --batch-size $BATCH --epochs 1 --lr 0.01 \
  --model-type resnet18 --momentum 0.9 > gpurun_out/cprof_b${BATCH}_e${ENGINE}.log 2>&1
python -c "import pstats; pstats.Stats('/tmp/ref.prof').sort_stats('tottime').print_stats(35)" > gpurun_out/cprof_b${BATCH}_e${ENGINE}.txt
python -c "import pstats; pstats.Stats('/tmp/ref.prof').sort_stats('cumulative').print_stats(45)" >> gpurun_out/cprof_b${BATCH}_e${ENGINE}.txt
