bash tools/gpu_steps.sh \
  tf_tests 400 "python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_gpu.py tests/test_comm_gpu.py" || exit 1
for m in vit_b_16 resnet152; do for v in 0 1; do
  timeout -k 10 200 python bench.py --model $m --steps 10 --warmup 3 --wgrad-stream $v > gpurun_out/models_${m}_$v.log 2>&1 || exit 1
  echo "$m wgrad_stream=$v $(grep '^{' gpurun_out/models_${m}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['loss_last'])")"
done; done
