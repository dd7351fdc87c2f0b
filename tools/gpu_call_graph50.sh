for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/g50_eager.log 2>&1 || exit 1
  echo "eager $(grep '^{' gpurun_out/g50_eager.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --graph > gpurun_out/g50_graph.log 2>&1 || exit 1
  echo "graph $(grep '^{' gpurun_out/g50_graph.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --wgrad-stream 0 > gpurun_out/g50_eager1.log 2>&1 || exit 1
  echo "eager-1stream $(grep '^{' gpurun_out/g50_eager1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
