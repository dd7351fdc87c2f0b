# weight-gradient side stream: correctness tests, then an A/B of the headline bench
bash tools/gpu_steps.sh \
  ws_tests 400 "python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_comm_gpu.py" || exit 1
for rep in 1 2; do for v in 0 1; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --wgrad-stream $v > gpurun_out/ws_bench_$v.log 2>&1 || exit 1
  echo "wgrad_stream=$v $(grep '^{' gpurun_out/ws_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
