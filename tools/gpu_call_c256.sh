for rep in 1 2; do for v in 96 200 400; do
  MI355X_DP_CONV256_MIN_TILES=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/c256_bench_$v.log 2>&1 || exit 1
  echo "min_tiles=$v $(grep '^{' gpurun_out/c256_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
