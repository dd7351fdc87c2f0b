export TMPDIR=/tmp
P="python3 tools/conv_probe.py --kind wgrad --N 256 --C 64 --H 56 --K 64 --R 3 --s 1 --iters 10"
timeout -k 10 120 $P > gpurun_out/probe_tn_time.log 2>&1 || exit 1
cat gpurun_out/probe_tn_time.log | grep wgrad
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmct1 -o run -- $P > gpurun_out/pmct1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d gpurun_out/pmct2 -o run -- $P > gpurun_out/pmct2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmct3 -o run -- $P > gpurun_out/pmct3.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmct_trace -o run -- $P > gpurun_out/pmct_trace.log 2>&1 || exit 1
