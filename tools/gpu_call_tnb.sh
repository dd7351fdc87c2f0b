for b in 512 1024 1536; do
  echo "== TN_BLOCKS $b"
  MI355X_DP_TN_BLOCKS=$b timeout -k 10 300 python tools/bench_conv.py --no-stock > gpurun_out/tnb_conv_$b.log 2>&1 || exit 1
  grep wgrad gpurun_out/tnb_conv_$b.log
  MI355X_DP_TN_BLOCKS=$b timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/tnb_bench_$b.log 2>&1 || exit 1
  grep '^{' gpurun_out/tnb_bench_$b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
