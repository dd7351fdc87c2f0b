# ResNet-152 / ViT-B/16 (BASELINE 8-GPU configs): with a process group, 8 vs 4 hardware queues
bash tools/gpu_steps.sh \
  m152_plain 200 "python bench.py --model resnet152 --steps 10 --warmup 3" \
  m152_force 200 "python bench.py --model resnet152 --steps 10 --warmup 3 --force-comm" \
  m152_force_q4 200 "MI355X_DP_HW_QUEUES=0 python bench.py --model resnet152 --steps 10 --warmup 3 --force-comm" \
  vit_plain 200 "python bench.py --model vit_b_16 --steps 10 --warmup 3" \
  vit_force 200 "python bench.py --model vit_b_16 --steps 10 --warmup 3 --force-comm" \
  vit_force_q4 200 "MI355X_DP_HW_QUEUES=0 python bench.py --model vit_b_16 --steps 10 --warmup 3 --force-comm"
