#!/bin/bash
# round 6: 1x1 weight gradients on the 256x256 TN GEMM (MI355X_DP_WGRAD256) -- test, isolated A/B,
# same-box step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/wg256
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -x \
  tests/test_gemm256_gpu.py > gpurun_out/r6/wg256/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/wg256/t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bench_wgrad256.py > gpurun_out/r6/wg256/iso.log 2>&1 || exit $?
cat gpurun_out/r6/wg256/iso.log
run() {
  local tag=$1 model=$2; shift 2
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model $model \
    > gpurun_out/r6/wg256/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/wg256/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run rn50_def_$r resnet50 || exit $?
  run rn50_w1_$r resnet50 MI355X_DP_WGRAD256=1 || exit $?
  run rn50_w4_$r resnet50 MI355X_DP_WGRAD256=4 || exit $?
done
for r in a b; do
  run r152_def_$r resnet152 || exit $?
  run r152_w1_$r resnet152 MI355X_DP_WGRAD256=1 || exit $?
  run r152_w4_$r resnet152 MI355X_DP_WGRAD256=4 || exit $?
done
