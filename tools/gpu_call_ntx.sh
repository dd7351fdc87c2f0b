export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  ntx_tests 600 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_resblock_gpu.py tests/test_comm_gpu.py" || exit 1
grep -q " passed" gpurun_out/ntx_tests.log && ! grep -q "failed" gpurun_out/ntx_tests.log || exit 1
for rep in 1 2; do for v in "" old; do
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ntx_bench_$v.log 2>&1 || exit 1
  echo "variant '$v' $(grep '^{' gpurun_out/ntx_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
P="python3 tools/conv_probe.py --kind dgrad --N 256 --C 128 --H 56 --K 128 --R 3 --s 2 --iters 10"
timeout -k 10 120 $P | grep dgrad
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcn3 -o run -- $P > gpurun_out/pmcn3.log 2>&1 || exit 1
MI355X_DP_KERNEL_VARIANT=old timeout -k 10 120 $P | grep dgrad
MI355X_DP_KERNEL_VARIANT=old timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcn3old -o run -- $P > gpurun_out/pmcn3old.log 2>&1 || exit 1
timeout -k 10 400 python tools/bench_conv.py --no-stock > gpurun_out/bench_conv_ntx.log 2>&1 || exit 1
grep "aggregate" gpurun_out/bench_conv_ntx.log
