#!/bin/bash
# round 6 end: full GPU suite, smoke(), steady-state ResNet-50 profile with every round-6 change
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/gpu_final.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r6/gpu_final.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6/smoke_final.log 2>&1 || exit $?
tail -2 gpurun_out/r6/smoke_final.log
MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 bash tools/r4_prof_grid.sh r6/r6_final || exit $?
head -12 gpurun_out/r6/r6_final.summary.md
