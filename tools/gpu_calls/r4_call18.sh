bash tools/gpu_steps_safe.sh \
 "r4_t18:400:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_stem_gpu.py tests/test_resblock_gpu.py tests/test_kernels_gpu.py -k 'stem or entropy or linear or resnet50_bs256 or resnet18_train or fused'" \
 "r4_bench_nol:300:python tools/bench_nol.py" \
 "r4_prof18:400:MI355X_DP_NOL=0 bash tools/r4_prof_grid.sh r4_p18"
