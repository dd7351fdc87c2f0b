python -c "import torch; print('priority_range', torch.cuda.Stream.priority_range()); s=torch.cuda.Stream(priority=1); print('p1 ->', s.priority); s=torch.cuda.Stream(priority=-1); print('p-1 ->', s.priority)"
for rep in 1 2; do for v in 0 1 3; do
  MI355X_DP_WGRAD_PRIORITY=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/prio_bench_$v.log 2>&1 || exit 1
  echo "priority=$v $(grep '^{' gpurun_out/prio_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
