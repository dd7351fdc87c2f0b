#!/bin/bash
# Profile the UNMODIFIED reference GPU script (staged in ref_fixture/ by build()) on one GPU:
# the SM_* / rank env a job would set is exported here, and the script itself runs right after
# rocprofv3's `--` (no launcher hop).  Outputs go to gpurun_out/refprof*.
#   bash tools/profile_reference_script.sh [EPOCHS]
set -e
EPOCHS=${1:-2}
export TMPDIR=/tmp
REPO=$(pwd)
mkdir -p gpurun_out /tmp/refmodel
python -c "import sys; sys.path.insert(0, '$REPO'); from mi355x_dp.data.cifar import write_synthetic_cifar10 as w; w('/tmp/refcifar')"
export SM_HOSTS='["algo-1"]' SM_CURRENT_HOST=algo-1 SM_MODEL_DIR=/tmp/refmodel SM_CHANNEL_TRAIN=/tmp/refcifar
export LOCAL_RANK=0 RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517
export PYTHONPATH=$REPO:$REPO/compat
SCRIPT=ref_fixture/notebooks/code/cifar10-distributed-smddp-gpu.py
ARGS="--backend smddp --batch-size 256 --epochs $EPOCHS --lr 0.01 --model-type resnet18 --momentum 0.9"
timeout -k 10 300 python -m cProfile -o gpurun_out/refprof_cprofile.out $SCRIPT $ARGS > gpurun_out/refprof_cprofile.log 2>&1
python -c "import pstats; pstats.Stats('gpurun_out/refprof_cprofile.out').sort_stats('tottime').print_stats(40)" > gpurun_out/refprof_cprofile.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/refprof_rocprof -o run -- python3 $SCRIPT $ARGS > gpurun_out/refprof_rocprof.log 2>&1
