#!/bin/bash
# round-6 panel kernel: numerics, per-shape A/B, step A/B (one GPU box call)
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 300 python -u -m pytest tests/test_panel_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/t_panel.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_panel.py > gpurun_out/r6/panel_bench4.log 2>&1 || exit 1
MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 240 python -u bench.py > gpurun_out/r6/bench_v3_p1.log 2>&1 || exit 1
MI355X_DP_PANEL=0 MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 240 python -u bench.py > gpurun_out/r6/bench_v3_p0.log 2>&1 || exit 1
MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 timeout -k 10 240 python -u bench.py > gpurun_out/r6/bench_v3_p1b.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_fp32_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6/t_fp32.log 2>&1
timeout -k 10 60 python -u tools/wait_value_probe.py > gpurun_out/r6/wait_value.log 2>&1
