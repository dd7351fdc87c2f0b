bash tools/gpu_steps.sh \
  bnfin_tests 600 "python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resblock_gpu.py tests/test_comm_gpu.py tests/test_trajectory_gpu.py" || exit 1
grep -q "rc=0" <(tail -3 gpurun_out/bnfin_tests.log) || true
for rep in 1 2; do for v in 0 1; do
  MI355X_DP_FUSED_BNFIN=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/bnfin_bench_$v.log 2>&1 || exit 1
  echo "fused_bnfin=$v $(grep '^{' gpurun_out/bnfin_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['loss_last'])")"
done; done
