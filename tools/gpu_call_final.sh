bash tools/gpu_steps.sh \
  mntd_train 300 "python tools/bench_mntd_train.py --device cuda --models 24 --epochs 3" \
  r18_graph_force 200 "python bench.py --model resnet18 --image-size 32 --batch 32 --graph --force-comm --steps 200 --warmup 5" \
  all_gpu_tests 900 "python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu" \
  bench 200 "python bench.py --steps 20 --warmup 5" \
  bench_force 200 "python bench.py --steps 20 --warmup 5 --force-comm"
