#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 300 python tools/bench_fold.py > gpurun_out/r6/bench_fold_ab.log 2>&1 || exit $?
cat gpurun_out/r6/bench_fold_ab.log
MI355X_DP_BN_FOLD=1 MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 bash tools/r4_prof_grid.sh r6/r6_fold || exit 1
MI355X_DP_BN_FOLD=0 MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 bash tools/r4_prof_grid.sh r6/r6_nofold || exit 1
head -8 gpurun_out/r6/r6_fold.summary.md; head -8 gpurun_out/r6/r6_nofold.summary.md
