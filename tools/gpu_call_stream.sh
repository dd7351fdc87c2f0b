export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  stream_tests 600 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_resblock_gpu.py tests/test_comm_gpu.py tests/test_trajectory_gpu.py" || exit 1
grep -q " passed" gpurun_out/stream_tests.log && ! grep -q "failed" gpurun_out/stream_tests.log || exit 1
for k in "fwd --N 256 --C 64 --H 56 --K 256 --R 1 --s 1" "dgrad --N 256 --C 256 --H 56 --K 64 --R 1 --s 1" "fwd --N 256 --C 128 --H 28 --K 512 --R 1 --s 1" "dgrad --N 256 --C 512 --H 28 --K 128 --R 1 --s 1"; do
  for v in 1 0; do
    echo "stream=$v $(MI355X_DP_NT_STREAM=$v timeout -k 10 60 python3 tools/conv_probe.py --kind $k --iters 20 2>&1 | grep TFLOP)"
  done
done
for rep in 1 2; do for v in 1 0; do
  MI355X_DP_NT_STREAM=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/stream_bench_$v.log 2>&1 || exit 1
  echo "stream=$v $(grep '^{' gpurun_out/stream_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
