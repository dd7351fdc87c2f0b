for rep in 1 2 3; do for v in 0 -1; do
  MI355X_DP_MAIN_PRIORITY=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/mprio_bench_$v.log 2>&1 || exit 1
  echo "main priority=$v $(grep '^{' gpurun_out/mprio_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
