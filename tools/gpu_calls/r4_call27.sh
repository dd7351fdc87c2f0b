bash tools/gpu_steps_safe.sh \
 "r4_conv_roof:400:python tools/bench_conv.py --model resnet50 --batch 256 --no-stock" \
 "r4_rn152:300:python bench.py --model resnet152 --steps 10 --warmup 3" \
 "r4_rn18g:300:python bench.py --model resnet18 --image-size 32 --batch 32 --graph --steps 100 --warmup 5" \
 "r4_prof27:400:bash tools/r4_prof_grid.sh r4_p27"
