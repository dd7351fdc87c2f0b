for rep in 1 2; do for v in 384 320 256 192 128; do
  MI355X_DP_TN_BLOCKS=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/tnb_bench_$v.log 2>&1 || exit 1
  echo "tn_blocks=$v $(grep '^{' gpurun_out/tnb_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
for v in 384 256; do
  MI355X_DP_TN_BLOCKS=$v timeout -k 10 200 python bench.py --model resnet152 --steps 10 --warmup 3 > gpurun_out/tnb_r152_$v.log 2>&1 || exit 1
  echo "r152 tn_blocks=$v $(grep '^{' gpurun_out/tnb_r152_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
