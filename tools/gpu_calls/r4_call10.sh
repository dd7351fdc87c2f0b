export TMPDIR=/tmp
bash tools/gpu_steps_safe.sh \
 "r4_hiptrace:200:rocprofv3 --hip-trace --kernel-trace -d gpurun_out/r4_hipt -o run -- python3 tools/graphed_comm_bench.py --mode gated --steps 40" || exit $?
db=$(find gpurun_out/r4_hipt -name '*results.db' | head -1)
python tools/hip_api_top.py $db > gpurun_out/r4_hip_api_top.md 2>&1
python tools/gate_timeline.py $db > gpurun_out/r4_hipt_timeline.txt 2>&1
rm -rf gpurun_out/r4_hipt
