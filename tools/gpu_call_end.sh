bash tools/gpu_steps.sh \
  end_smoke 300 "python -c 'import __graft_entry__ as g; g.smoke()'" \
  end_gpu_tests 900 "python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu" \
  end_bench 200 "python bench.py --gpus 1 --steps 20 --warmup 5"
