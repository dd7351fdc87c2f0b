export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf1 -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmcf1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcf2 -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmcf2.log 2>&1 || exit 1
