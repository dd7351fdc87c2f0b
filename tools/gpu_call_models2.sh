export TMPDIR=/tmp
for m in resnet152 vit_b_16; do
  timeout -k 10 200 python bench.py --model $m --steps 20 --warmup 5 > gpurun_out/m2_$m.log 2>&1 || exit 1
  grep '^{' gpurun_out/m2_$m.log
done
timeout -k 10 200 python bench.py --model resnet18 --batch 32 --image-size 32 --num-classes 10 --steps 200 --warmup 5 --graph > gpurun_out/m2_r18g.log 2>&1 || exit 1
grep '^{' gpurun_out/m2_r18g.log
timeout -k 10 200 python bench.py --model resnet18 --batch 32 --image-size 32 --num-classes 10 --steps 200 --warmup 5 > gpurun_out/m2_r18e.log 2>&1 || exit 1
grep '^{' gpurun_out/m2_r18e.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r152 -o run -- python3 bench.py --model resnet152 --steps 6 --warmup 2 > gpurun_out/prof_r152.log 2>&1 || exit 1
