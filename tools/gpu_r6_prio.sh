#!/bin/bash
# round 6: compute stream at high priority (its workgroups dispatched ahead of the weight-gradient side
# stream's) -- same box, interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/prio
run() {
  local tag=$1 model=$2; shift 2
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model $model \
    > gpurun_out/r6/prio/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/prio/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run rn50_def_$r resnet50 || exit $?
  run rn50_main_$r resnet50 MI355X_DP_MAIN_PRIORITY=-1 || exit $?
  run rn50_side_$r resnet50 MI355X_DP_WGRAD_PRIORITY=-1 || exit $?
done
for r in a b; do
  run r152_def_$r resnet152 || exit $?
  run r152_main_$r resnet152 MI355X_DP_MAIN_PRIORITY=-1 || exit $?
done
