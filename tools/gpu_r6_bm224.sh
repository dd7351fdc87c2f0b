#!/bin/bash
# round 6: 224-row tiles in the 256-wide NT kernel -- tests (forced 224 / 256, auto choice), then
# same-box A/Bs: ResNet-50, ResNet-152, ViT-B/16 with MI355X_DP_G256_BM224=1 (auto) vs 0
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6/bm224
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -x \
  tests/test_gemm256_gpu.py tests/test_graph_workspaces_gpu.py tests/test_transformer_gpu.py \
  tests/test_kernels_gpu.py::test_resnet50_bs256_train_step_matches_fp32 > gpurun_out/r6/bm224/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6/bm224/t.log
[ $rc -eq 0 ] || exit $rc
run() {  # tag model env...
  local tag=$1 model=$2; shift 2
  env "$@" MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py --model $model \
    > gpurun_out/r6/bm224/$tag.log 2>&1 || return $?
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r6/bm224/$tag.log') if l.startswith('{')][-1]); print('$tag', d['value'], d['ms_per_step'])"
}
for r in a b; do
  run rn50_auto_$r resnet50 MI355X_DP_G256_BM224=1 || exit $?
  run rn50_off_$r resnet50 MI355X_DP_G256_BM224=0 || exit $?
done
for r in a b; do
  run r152_auto_$r resnet152 MI355X_DP_G256_BM224=1 || exit $?
  run r152_off_$r resnet152 MI355X_DP_G256_BM224=0 || exit $?
done
for r in a; do
  run vit_auto_$r vit_b_16 MI355X_DP_G256_BM224=1 || exit $?
  run vit_off_$r vit_b_16 MI355X_DP_G256_BM224=0 || exit $?
done
