#!/bin/bash
# RN50 bs256 profile: steady-state kernel summary + per-launch-shape attribution (+ the GEMM/conv
# geometry of every launch from MI355X_DP_TRACE_GEMM=1), then per-shape conv timings at 1 and 2
# NT stages.
export TMPDIR=/tmp
mkdir -p gpurun_out
name=${1:-r4_rn50}
shift
timeout -k 10 300 env MI355X_DP_TRACE_GEMM=1 rocprofv3 --kernel-trace --stats -d gpurun_out/$name -o run -- python3 bench.py --steps 6 --warmup 3 "$@" > gpurun_out/$name.bench.log 2> gpurun_out/$name.trace.err || exit $?
db=$(find gpurun_out/$name -name '*results.db' | head -1)
python tools/prof_summary.py $db --marker sgd_flat_kernel --skip 4 > gpurun_out/$name.summary.md
python tools/prof_by_grid.py $db --marker sgd_flat_kernel --skip 4 --top 80 > gpurun_out/$name.grid.md
python tools/prof_neighbors.py $db --marker sgd_flat_kernel --step 5 > gpurun_out/$name.neighbors.txt
python tools/prof_sequence.py $db --marker sgd_flat_kernel --step 5 > gpurun_out/$name.seq.txt
grep "^\[gemm\]" gpurun_out/$name.trace.err | sort -u > gpurun_out/$name.gemm_shapes.txt
rm -rf gpurun_out/$name
