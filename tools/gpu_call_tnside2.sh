for rep in 1 2; do for v in 384 256 512 640; do
  MI355X_DP_TN_BLOCKS_SIDE=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/tns2_$v.log 2>&1 || exit 1
  echo "side_blocks=$v $(grep '^{' gpurun_out/tns2_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
