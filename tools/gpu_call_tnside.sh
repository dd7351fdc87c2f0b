for rep in 1 2; do for v in default 768 384; do
  if [ $v = default ]; then unset MI355X_DP_TN_BLOCKS_SIDE; else export MI355X_DP_TN_BLOCKS_SIDE=$v; fi
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/tnside_$v.log 2>&1 || exit 1
  echo "side=$v $(grep '^{' gpurun_out/tnside_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
unset MI355X_DP_TN_BLOCKS_SIDE
MI355X_DP_TRACE_GEMM=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 > gpurun_out/tnside_trace.log 2>&1 || exit 1
grep "tn128x128" gpurun_out/tnside_trace.log | head -8
