# what does a process group cost at N=1?  plain vs force-comm (nccl hi-prio / normal prio / smddp), then kernel traces
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  pg_plain 150 "python bench.py --steps 20 --warmup 5" \
  pg_nccl 150 "python bench.py --steps 20 --warmup 5 --force-comm" \
  pg_nccl_lo 150 "MI355X_DP_NCCL_HIPRIO=0 python bench.py --steps 20 --warmup 5 --force-comm" \
  pg_smddp 150 "python bench.py --steps 20 --warmup 5 --force-comm --backend smddp" \
  pg_nccl_ws0 150 "python bench.py --steps 20 --warmup 5 --force-comm --wgrad-stream 0" \
  pg_plain_ws0 150 "python bench.py --steps 20 --warmup 5 --wgrad-stream 0" \
  prof_plain 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_plain -o run -- python3 bench.py --steps 10 --warmup 3" \
  prof_nccl 200 "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_nccl -o run -- python3 bench.py --steps 10 --warmup 3 --force-comm"
