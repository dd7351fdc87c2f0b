export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  swz_tests 600 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm256_gpu.py tests/test_resblock_gpu.py" || exit 1
grep -q " passed" gpurun_out/swz_tests.log && ! grep -q "failed" gpurun_out/swz_tests.log || exit 1
for rep in 1 2; do for v in "" noswz; do
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/swz_bench_$v.log 2>&1 || exit 1
  echo "variant '$v' $(grep '^{' gpurun_out/swz_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
for v in "" noswz; do
  MI355X_DP_KERNEL_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d gpurun_out/pmc_swz$v -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc_swz$v.log 2>&1 || exit 1
done
timeout -k 10 400 python tools/bench_conv.py --no-stock > gpurun_out/bench_conv.log 2>&1 || exit 1
tail -5 gpurun_out/bench_conv.log
