# HBM bytes per RN50 step (two counter passes), then ViT with/without the library data-gradient GEMMs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcF -o run -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/r4_pmcF.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcW -o run -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/r4_pmcW.log 2>&1 &&
python tools/pmc_bytes.py --fetch $(find gpurun_out/pmcF -name '*counter_collection.csv' | head -1) --write $(find gpurun_out/pmcW -name '*counter_collection.csv' | head -1) --ms-per-step 20.5 > gpurun_out/r4_pmc_bytes.md &&
rm -rf gpurun_out/pmcF gpurun_out/pmcW &&
bash tools/gpu_steps_safe.sh \
 "r4_vit_lib:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_vit_native:300:MI355X_DP_BLAS_DGRAD=0 python bench.py --model vit_b_16 --steps 10 --warmup 3"
