for rep in 1 2; do for v in "" rw4 rw8; do
  MI355X_DP_KERNEL_VARIANT=$v timeout -k 10 200 python bench.py --model vit_b_16 --steps 10 --warmup 3 > gpurun_out/lnrw_$v.log 2>&1 || exit 1
  echo "variant '$v' $(grep '^{' gpurun_out/lnrw_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done; done
