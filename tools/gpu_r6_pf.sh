#!/bin/bash
# round 6: 32-column panels (K up to 1024) -- panel tests, then same-box A/B of panel-before-256-wide
# routing (MI355X_DP_PANEL_FIRST) and of the layer-2 fold (MI355X_DP_BN_FOLD_MAXK=512)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/pf
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -x \
  tests/test_panel_gpu.py > gpurun_out/r6/pf/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/pf/t.log
[ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1 model=$2; shift 2
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model $model \
    > gpurun_out/r6/pf/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/pf/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run rn50_def_$r resnet50 || exit $?
  run rn50_pf_$r resnet50 MI355X_DP_PANEL_FIRST=1 || exit $?
  run rn50_f512_$r resnet50 MI355X_DP_BN_FOLD_MAXK=512 || exit $?
done
for r in a b; do
  run r152_def_$r resnet152 || exit $?
  run r152_pf_$r resnet152 MI355X_DP_PANEL_FIRST=1 || exit $?
done
