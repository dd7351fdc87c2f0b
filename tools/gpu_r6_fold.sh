#!/bin/bash
# round 6: folded BN backward -- kernel tests, block test, bench-config gradient test, then a same-box
# A/B of the ResNet-50 step (MI355X_DP_BN_FOLD=1 / 0 / 1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -x \
  tests/test_panel_gpu.py tests/test_resblock_gpu.py::test_folded_bn_backward_matches_materialised \
  "tests/test_fp32_gpu.py::test_f32_batchnorm_train" \
  tests/test_kernels_gpu.py::test_resnet50_bs256_train_step_matches_fp32 > gpurun_out/r6/t_fold.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r6/t_fold.log
[ $rc -eq 0 ] || exit $rc
for tag in 1 0 1b; do
  v=${tag:0:1}
  MI355X_DP_BN_FOLD=$v MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py \
    > gpurun_out/r6/bench_fold$tag.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r6/bench_fold$tag.log') if l.startswith('{')][-1]); print('fold=$tag', d['value'], d['ms_per_step'])"
done
