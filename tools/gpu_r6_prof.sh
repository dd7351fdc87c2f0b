#!/bin/bash
# round-6 steady-state ResNet-50 profile (panel kernels on) + ResNet-152 / ViT benches
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 bash tools/r4_prof_grid.sh r6/r6_rn50 || exit 1
