set -o pipefail
mkdir -p gpurun_out
for m in nocomm ungated gated; do
  timeout -k 10 120 python tools/graphed_comm_bench.py --mode $m >> gpurun_out/r4_gate_ab.log 2>&1 || exit $?
done
for m in ungated gated; do
  timeout -k 10 120 python tools/graphed_comm_bench.py --mode $m --backend nccl >> gpurun_out/r4_gate_ab.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_gate_prof -o run -- python3 tools/graphed_comm_bench.py --mode gated --steps 50 >> gpurun_out/r4_gate_ab.log 2>&1
db=$(find gpurun_out/r4_gate_prof -name '*results.db' | head -1)
python tools/prof_summary.py $db > gpurun_out/r4_gate_prof.summary.md
python tools/gate_timeline.py $db > gpurun_out/r4_gate_timeline.txt
rm -rf gpurun_out/r4_gate_prof
