for v in "" tn4 n6 n6tn4; do
  echo "== variant '$v'"
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 300 python tools/bench_conv.py --no-stock > gpurun_out/ab3_conv_$v.log 2>&1 || exit 1
  grep "ms per step" gpurun_out/ab3_conv_$v.log
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/ab3_bench_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab3_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
