#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider -x \
  tests/test_panel_gpu.py tests/test_resblock_gpu.py \
  tests/test_kernels_gpu.py::test_resnet50_bs256_train_step_matches_fp32 > gpurun_out/r6/t_fold3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r6/t_fold3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_fold.py > gpurun_out/r6/bench_fold_ab4.log 2>&1 || exit $?
cat gpurun_out/r6/bench_fold_ab4.log
for tag in 1 0 1b 0b; do
  v=${tag:0:1}
  MI355X_DP_BN_FOLD=$v MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 200 python bench.py \
    > gpurun_out/r6/bench_f4_$tag.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r6/bench_f4_$tag.log') if l.startswith('{')][-1]); print('fold=$tag', d['value'], d['ms_per_step'])"
done
