r() { echo "== $*" >> gpurun_out/r4_gate_ab4.log; timeout -k 10 120 env "$@" python tools/graphed_comm_bench.py --mode gated >> gpurun_out/r4_gate_ab4.log 2>&1; }
mkdir -p gpurun_out
r A=1 && r MI355X_DP_GATE_PRIO=-1 && r MI355X_DP_SMDDP_HIPRIO=0 && r MI355X_DP_GATE_DEBUG=after MI355X_DP_SMDDP_HIPRIO=0 && timeout -k 10 120 python tools/graphed_comm_bench.py --mode ungated >> gpurun_out/r4_gate_ab4.log 2>&1
