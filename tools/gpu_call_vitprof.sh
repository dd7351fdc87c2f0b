export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit2 -o run -- python3 bench.py --model vit_b_16 --steps 6 --warmup 2 > gpurun_out/prof_vit2.log 2>&1 || exit 1
grep '^{' gpurun_out/prof_vit2.log | cut -c1-150
