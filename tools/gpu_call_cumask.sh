for rep in 1 2; do for v in 0 8 16 32 64; do
  MI355X_DP_WGRAD_RESERVE_CUS=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/cumask_bench_$v.log 2>&1 || exit 1
  echo "reserve=$v $(grep '^{' gpurun_out/cumask_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
