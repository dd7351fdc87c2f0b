for rep in 1 2; do for v in "" k64; do
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/k64_bench_$v.log 2>&1 || exit 1
  echo "variant '$v' $(grep '^{' gpurun_out/k64_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
MI355X_DP_KERNEL_VARIANT=k64 timeout -k 10 400 python tools/bench_conv.py --no-stock > gpurun_out/bench_conv_k64.log 2>&1 || exit 1
grep "256 64 56 256\|256 64 56 64 1\|256 128 28 512\|aggregate" gpurun_out/bench_conv_k64.log
