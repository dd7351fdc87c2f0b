bash tools/gpu_steps.sh conv_tests 500 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_resblock_gpu.py" || exit 1
for v in "" o3; do
  echo "== variant '$v'"
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 300 python tools/bench_conv.py --no-stock > gpurun_out/occ_conv_$v.log 2>&1 || exit 1
  grep "ms per step" gpurun_out/occ_conv_$v.log
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/occ_bench_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/occ_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
