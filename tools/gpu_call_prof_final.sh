export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_final.log 2>&1 || exit 1
grep '^{' gpurun_out/prof_final.log | cut -c1-200
