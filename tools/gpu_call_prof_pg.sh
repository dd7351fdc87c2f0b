export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  prof_pg8 240 "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pg8 -o run -- python3 bench.py --steps 10 --warmup 3 --force-comm"
