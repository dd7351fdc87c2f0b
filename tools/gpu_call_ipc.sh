bash tools/gpu_steps.sh \
  ipc_tests 400 "python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_integration.py -k 'ipc or smddp' tests/test_comm_gpu.py" \
  ipc_overlap 360 "bash tools/rehearse_ipc_overlap.sh resnet50 64 6"
