bash tools/gpu_steps.sh \
  ds_tests 600 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_comm_gpu.py tests/test_resblock_gpu.py tests/test_graphs_gpu.py tests/test_gemm256_gpu.py" || exit 1
grep -q " passed" gpurun_out/ds_tests.log && ! grep -q "failed" gpurun_out/ds_tests.log || exit 1
for rep in 1 2; do for v in 0 1; do
  MI355X_DP_DS_STREAM=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ds_bench_$v.log 2>&1 || exit 1
  echo "ds_stream=$v $(grep '^{' gpurun_out/ds_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
