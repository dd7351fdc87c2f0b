# side-stream priority A/B, then a kernel trace of the default configuration
for rep in 1 2; do for v in 0 -1; do
  MI355X_DP_WGRAD_PRIORITY=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/prio_bench_$v.log 2>&1 || exit 1
  echo "priority=$v $(grep '^{' gpurun_out/prio_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ws -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_ws.log 2>&1 || exit 1
grep '^{' gpurun_out/prof_ws.log
timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_integration.py -k debug_kernels > gpurun_out/dbg_tests.log 2>&1; echo "debug test rc=$?"; tail -3 gpurun_out/dbg_tests.log
