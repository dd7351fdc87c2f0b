#!/bin/bash
# round 6 end: full GPU suite, smoke(), steady-state ResNet-50 profile with every round-6 change
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6/gpu_final2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r6/gpu_final2.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6/smoke_final2.log 2>&1 || exit $?
tail -2 gpurun_out/r6/smoke_final2.log
MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 bash tools/r4_prof_grid.sh r6/r6_final2 || exit $?
head -12 gpurun_out/r6/r6_final2.summary.md
run() {
  local tag=$1; shift
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py \
    > gpurun_out/r6/final_$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/final_$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run rn50_def_$r || exit $?
  run rn50_side512_$r MI355X_DP_TN_BLOCKS_SIDE=512 || exit $?
done
