#!/bin/bash
# Profile the UNMODIFIED reference GPU script (staged in ref_fixture/ by build()) on one GPU:
# the SM_* / rank env a job would set is exported here, and the script itself runs right after
# rocprofv3's `--` (no launcher hop).  Outputs go to gpurun_out/refprof_<TAG>*.
#   bash tools/profile_reference_script.sh [EPOCHS] [BATCH] [ENGINE_DDP 1|0] [TAG]
# BATCH 32 is the per-rank shape of the reference's 8-GPU job (gpu.py:122-124: 256 // 8);
# ENGINE_DDP=0 keeps torch's stock DistributedDataParallel (MI355X_DP_ENGINE_DDP).
set -e
EPOCHS=${1:-2}
BATCH=${2:-256}
ENGINE=${3:-1}
TAG=${4:-b${BATCH}_e${ENGINE}}
export TMPDIR=/tmp
REPO=$(pwd)
mkdir -p gpurun_out /tmp/refmodel_$TAG
python -c "import sys; sys.path.insert(0, '$REPO'); from mi355x_dp.data.cifar import write_synthetic_cifar10 as w; w('/tmp/refcifar')"
export SM_HOSTS='["algo-1"]' SM_CURRENT_HOST=algo-1 SM_MODEL_DIR=/tmp/refmodel_$TAG SM_CHANNEL_TRAIN=/tmp/refcifar
export LOCAL_RANK=0 RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517
export PYTHONPATH=$REPO:$REPO/compat MI355X_DP_ENGINE_DDP=$ENGINE
SCRIPT=ref_fixture/notebooks/code/cifar10-distributed-smddp-gpu.py
ARGS="--backend smddp --batch-size $BATCH --epochs $EPOCHS --lr 0.01 --model-type resnet18 --momentum 0.9"
start=$(date +%s.%N)
timeout -k 10 400 python3 $SCRIPT $ARGS > gpurun_out/refprof_${TAG}_plain.log 2>&1
end=$(date +%s.%N)
echo "wall_s $(python -c "print(round($end - $start, 2))") epochs $EPOCHS batch $BATCH engine $ENGINE" | tee gpurun_out/refprof_${TAG}_wall.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/refprof_${TAG} -o run -- python3 $SCRIPT $ARGS > gpurun_out/refprof_${TAG}_rocprof.log 2>&1
# keep the summary (span, GPU busy, per-kernel table), drop the database (too large to copy back)
python tools/prof_summary.py $(find gpurun_out/refprof_${TAG} -name '*results.db' | head -1) --steps $((50000 / BATCH * EPOCHS)) \
  --title "unmodified cifar10-distributed-smddp-gpu.py, batch $BATCH, engine DDP $ENGINE" > gpurun_out/refprof_${TAG}.summary.md
rm -rf gpurun_out/refprof_${TAG}
