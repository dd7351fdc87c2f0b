bash tools/gpu_steps.sh aug_tests 300 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k 'augment or resnet18_train or conv_fwd'" || exit 1
grep -q " passed" gpurun_out/aug_tests.log && ! grep -q "failed" gpurun_out/aug_tests.log || exit 1
for rep in 1 2; do for v in "" old; do
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/aug_bench_$v.log 2>&1 || exit 1
  echo "variant '$v' $(grep '^{' gpurun_out/aug_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
