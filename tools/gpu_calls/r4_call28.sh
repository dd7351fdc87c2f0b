bash tools/gpu_steps_safe.sh \
 "r4_vws1_a:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_vws0_a:300:python bench.py --model vit_b_16 --steps 10 --warmup 3 --wgrad-stream 0" \
 "r4_vws1_b:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_vws0_b:300:python bench.py --model vit_b_16 --steps 10 --warmup 3 --wgrad-stream 0" \
 "r4_r152ws0:300:python bench.py --model resnet152 --steps 10 --warmup 3 --wgrad-stream 0"
