for rep in 1 2; do for v in 1 0; do
  MI355X_DP_GLDS=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/tn2_bench_$v.log 2>&1 || exit 1
  echo "tn_single_stage=$v $(grep '^{' gpurun_out/tn2_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
for v in 1 0; do for tb in 384 768; do
  MI355X_DP_GLDS=$v MI355X_DP_TN_BLOCKS_SIDE=$tb timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/tn2b_$v$tb.log 2>&1 || exit 1
  echo "tn_single_stage=$v side_blocks=$tb $(grep '^{' gpurun_out/tn2b_$v$tb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
MI355X_DP_GLDS=0 timeout -k 10 400 python tools/bench_conv.py --no-stock > gpurun_out/bench_conv_tn2.log 2>&1 || exit 1
grep "aggregate" gpurun_out/bench_conv_tn2.log
