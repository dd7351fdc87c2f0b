bash tools/gpu_steps.sh \
  all_gpu_tests 900 "python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu" \
  bench 200 "python bench.py --steps 20 --warmup 5" \
  bench_force 200 "python bench.py --steps 20 --warmup 5 --force-comm" \
  bench_force_shard 200 "python bench.py --steps 20 --warmup 5 --force-comm --shard-optimizer"
