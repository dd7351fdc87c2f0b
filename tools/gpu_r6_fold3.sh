#!/bin/bash
# round 6: folded BN backward on the 256-wide kernel (layer-3 expansions) -- tests, then same-box A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/fold3
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -x \
  tests/test_panel_gpu.py tests/test_gemm256_gpu.py tests/test_resblock_gpu.py \
  tests/test_kernels_gpu.py::test_resnet50_bs256_train_step_matches_fp32 > gpurun_out/r6/fold3/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/fold3/t.log
[ $rc -eq 0 ] || exit $rc
run() {  # tag model env...
  local tag=$1 model=$2; shift 2
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 MI355X_DP_TRACE_GEMM=1 timeout -k 10 200 python bench.py --model $model \
    > gpurun_out/r6/fold3/$tag.log 2> gpurun_out/r6/fold3/$tag.err || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/fold3/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run rn50_new_$r resnet50 || exit $?
  run rn50_l1only_$r resnet50 MI355X_DP_BN_FOLD_MAXK=256 || exit $?
done
for r in a b; do
  run r152_new_$r resnet152 || exit $?
  run r152_l1only_$r resnet152 MI355X_DP_BN_FOLD_MAXK=256 || exit $?
done
grep -h "g256dgrad-fbb" gpurun_out/r6/fold3/rn50_new_a.err | sort -u | head
