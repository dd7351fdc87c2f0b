#!/bin/bash
# round 6: layer-2 folded BN backward (32-column panels, MI355X_DP_BN_FOLD_MAXK=512) on ResNet-152 -- same box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/f512
run() {
  local tag=$1 model=$2; shift 2
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model $model \
    > gpurun_out/r6/f512/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/f512/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b c; do
  run r152_def_$r resnet152 || exit $?
  run r152_f512_$r resnet152 MI355X_DP_BN_FOLD_MAXK=512 || exit $?
done
