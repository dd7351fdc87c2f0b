#!/bin/bash
# round 6: stride-2 1x1 shortcut data gradients on the 256-wide kernel with scattered rows
# (MI355X_DP_DS256) -- tests, then same-box step A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/ds256
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -x \
  tests/test_gemm256_gpu.py tests/test_resblock_gpu.py tests/test_kernels_gpu.py > gpurun_out/r6/ds256/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/ds256/t.log
[ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1 model=$2; shift 2
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model $model \
    > gpurun_out/r6/ds256/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/ds256/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b c; do
  run rn50_on_$r resnet50 || exit $?
  run rn50_off_$r resnet50 MI355X_DP_DS256=0 || exit $?
done
for r in a b; do
  run r152_on_$r resnet152 || exit $?
  run r152_off_$r resnet152 MI355X_DP_DS256=0 || exit $?
done
