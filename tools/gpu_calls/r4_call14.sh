bash tools/gpu_steps_safe.sh \
 "r4_nol_tests:400:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_resblock_gpu.py tests/test_kernels_gpu.py -k 'resblock or fused or normalize or resnet50_bs256 or conv'" \
 "r4_nol_a0:200:MI355X_DP_NOL=0 python bench.py --steps 20 --warmup 5" \
 "r4_nol_b0:200:python bench.py --steps 20 --warmup 5" \
 "r4_nol_a1:200:MI355X_DP_NOL=0 python bench.py --steps 20 --warmup 5" \
 "r4_nol_b1:200:python bench.py --steps 20 --warmup 5" \
 "r4_bench_tn:300:python tools/bench_tn.py"
