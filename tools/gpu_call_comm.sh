bash tools/gpu_steps.sh \
  comm_tests 400 "python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_comm_gpu.py tests/test_gpu_integration.py" \
  prof_force_smddp 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_force_smddp -o run -- python3 bench.py --steps 5 --warmup 3 --force-comm --backend smddp" \
  prof_force_nccl 300 "rocprofv3 --kernel-trace --stats -d gpurun_out/prof_force_nccl -o run -- python3 bench.py --steps 5 --warmup 3 --force-comm --backend nccl"
