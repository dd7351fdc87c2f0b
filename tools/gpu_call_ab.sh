# A/B kernel-variant sweep: bench_bn summary + the ResNet-50 bench per variant
for v in "" g64k g16knts g64knts u1 u8g; do
  echo "== variant '$v'"
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 120 python tools/bench_bn.py > gpurun_out/ab_bn_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_bn_$v.log
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_bench_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
