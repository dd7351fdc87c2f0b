#!/bin/bash
# panel routing for every row count (MI355X_DP_PANEL=2: layer 4's M = 12,544 shapes too) vs default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/knobs2
run() {
  local tag=$1 model=$2; shift 2
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model $model \
    > gpurun_out/r6/knobs2/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/knobs2/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run rn50_def_$r resnet50 MI355X_DP_PANEL=1 || exit $?
  run rn50_p2_$r resnet50 MI355X_DP_PANEL=2 || exit $?
done
for r in a; do
  run r152_def_$r resnet152 MI355X_DP_PANEL=1 || exit $?
  run r152_p2_$r resnet152 MI355X_DP_PANEL=2 || exit $?
done
