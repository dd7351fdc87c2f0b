for rep in 1 2; do for v in 0 1; do
  MI355X_DP_DS_STREAM=$v timeout -k 10 120 python bench.py --model resnet18 --batch 32 --image-size 32 --num-classes 10 --steps 50 --warmup 5 > gpurun_out/ds2_bench_$v.log 2>&1 || exit 1
  echo "r18 bs32 ds_stream=$v $(grep '^{' gpurun_out/ds2_bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  MI355X_DP_DS_STREAM=$v timeout -k 10 120 python bench.py --model resnet50 --batch 64 --steps 30 --warmup 5 > gpurun_out/ds2_b64_$v.log 2>&1 || exit 1
  echo "r50 bs64 ds_stream=$v $(grep '^{' gpurun_out/ds2_b64_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
