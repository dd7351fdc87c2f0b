export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r4_vitp -o run -- python3 bench.py --model vit_b_16 --steps 6 --warmup 3 > gpurun_out/r4_vitp.bench.log 2> gpurun_out/r4_vitp.trace.err &&
db=$(find gpurun_out/r4_vitp -name '*results.db' | head -1) &&
python tools/prof_summary.py $db --marker sgd_flat_kernel --skip 4 > gpurun_out/r4_vitp.summary.md &&
python tools/prof_by_grid.py $db --marker sgd_flat_kernel --skip 4 --top 60 > gpurun_out/r4_vitp.grid.md &&
rm -rf gpurun_out/r4_vitp
