mkdir -p gpurun_out
timeout -k 10 120 python tools/graphed_comm_bench.py --mode gated >> gpurun_out/r4_gate_ab5.log 2>&1 && timeout -k 10 120 python tools/graphed_comm_bench.py --mode ungated >> gpurun_out/r4_gate_ab5.log 2>&1 && timeout -k 10 120 python tools/graphed_comm_bench.py --mode nocomm >> gpurun_out/r4_gate_ab5.log 2>&1
