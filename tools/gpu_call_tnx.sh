export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  tnx_tests 600 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_comm_gpu.py tests/test_transformer_gpu.py tests/test_gemm256_gpu.py" || exit 1
grep -q " passed" gpurun_out/tnx_tests.log && ! grep -q "failed" gpurun_out/tnx_tests.log || exit 1
for rep in 1 2; do for v in "" old; do
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/tnx_bench_$v.log 2>&1 || exit 1
  echo "variant '$v' $(grep '^{' gpurun_out/tnx_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
P="python3 tools/conv_probe.py --kind wgrad --N 256 --C 64 --H 56 --K 64 --R 3 --s 1 --iters 10"
timeout -k 10 120 $P | grep wgrad
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcx3 -o run -- $P > gpurun_out/pmcx3.log 2>&1 || exit 1
timeout -k 10 400 python tools/bench_conv.py --no-stock > gpurun_out/bench_conv_tnx.log 2>&1 || exit 1
grep "aggregate" gpurun_out/bench_conv_tnx.log
