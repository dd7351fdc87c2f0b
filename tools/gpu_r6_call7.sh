#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_engine_graph_gpu.py::test_graphed_comm_modes_match_eager tests/test_fp32_gpu.py \
  tests/test_kernels_gpu.py::test_normalize_on_load_kernels tests/test_panel_gpu.py \
  tests/test_comm_gpu.py > gpurun_out/r6/t_fix.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/r6/t_fix.log
bash tools/gpu_r6_w2trace.sh > gpurun_out/r6/w2trace.txt 2>&1; echo "w2trace rc=$?"; tail -20 gpurun_out/r6/w2trace.txt
bash tools/gpu_r6_prof.sh > gpurun_out/r6/prof.txt 2>&1; echo "prof rc=$?"; tail -5 gpurun_out/r6/prof.txt
