export TMPDIR=/tmp
P="python3 tools/conv_probe.py --kind fwd --N 256 --C 64 --H 56 --K 256 --R 1 --s 1 --iters 10"
timeout -k 10 120 $P > gpurun_out/probe_time.log 2>&1 || exit 1
cat gpurun_out/probe_time.log
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmcs1 -o run -- $P > gpurun_out/pmcs1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcs2 -o run -- $P > gpurun_out/pmcs2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcs3 -o run -- $P > gpurun_out/pmcs3.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcs_trace -o run -- $P > gpurun_out/pmcs_trace.log 2>&1 || exit 1
