set -o pipefail
mkdir -p gpurun_out
r() { echo "== $*" >> gpurun_out/r4_gate_ab2.log; timeout -k 10 120 env "$@" python tools/graphed_comm_bench.py --mode gated >> gpurun_out/r4_gate_ab2.log 2>&1; }
r A=1 && r MI355X_DP_GATE_DEBUG=nokernel && r MI355X_DP_GATE_DEBUG=after && r MI355X_DP_HW_QUEUES=16 && r MI355X_DP_SMDDP_HIPRIO=0 && timeout -k 10 120 python tools/graphed_comm_bench.py --mode ungated >> gpurun_out/r4_gate_ab2.log 2>&1
