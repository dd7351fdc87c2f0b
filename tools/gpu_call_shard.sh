# balanced-shard mode: GPU tests (IPC mesh RS/AG on 2 ranks sharing the GPU, RCCL/smddp RS/AG at world 1)
bash tools/gpu_steps.sh \
  shard_tests 400 "python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_integration.py::test_smddp_ipc_balanced_shards_two_ranks tests/test_comm_gpu.py::test_force_comm_world1_shard_optimizer tests/test_gpu_integration.py::test_smddp_ipc_only_two_ranks" \
  rn50_grad 300 "python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_kernels_gpu.py::test_resnet50_bs256_train_step_matches_fp32" \
  bench_shard 200 "python bench.py --steps 20 --warmup 5 --force-comm --shard-optimizer" \
  bench_force 200 "python bench.py --steps 20 --warmup 5 --force-comm"
