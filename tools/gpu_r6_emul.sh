#!/bin/bash
# round 6: the default bench line (ResNet-152 / ViT secondaries + emulated 8-rank comm), then a
# kernel trace of the emulated-comm step (ring_emulate_kernel on the smddp comm stream under backward)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
timeout -k 10 600 python bench.py > gpurun_out/r6/bench_default.log 2>&1 || exit $?
tail -1 gpurun_out/r6/bench_default.log | cut -c1-600
name=r6/r6_emul
timeout -k 10 300 env MI355X_DP_BENCH_SECONDARY=0 MI355X_DP_BENCH_EMULATE=0 rocprofv3 --kernel-trace --stats \
  -d gpurun_out/$name -o run -- python3 bench.py --comm-emulate 8 --steps 6 --warmup 3 \
  > gpurun_out/$name.bench.log 2> gpurun_out/$name.trace.err || exit $?
db=$(find gpurun_out/$name -name '*results.db' | head -1)
python tools/prof_summary.py $db --marker sgd_flat_kernel --skip 4 > gpurun_out/$name.summary.md
python tools/prof_sequence.py $db --marker sgd_flat_kernel --step 5 > gpurun_out/$name.seq.txt
rm -rf gpurun_out/$name
head -12 gpurun_out/$name.summary.md
