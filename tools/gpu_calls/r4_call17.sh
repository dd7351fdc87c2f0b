bash tools/gpu_steps_safe.sh \
 "r4_nol_tests2:500:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resblock_gpu.py tests/test_kernels_gpu.py -k 'resblock or fused or normalize or resnet50_bs256 or resnet18_train'" \
 "r4_prof_nol0:400:MI355X_DP_NOL=0 bash tools/r4_prof_grid.sh r4_nol0" \
 "r4_prof_nol1:400:bash tools/r4_prof_grid.sh r4_nol1" &&
bash tools/gpu_steps_safe.sh \
 "r4_nolab_a0:200:MI355X_DP_NOL=0 python bench.py --steps 20 --warmup 5" \
 "r4_nolab_b0:200:python bench.py --steps 20 --warmup 5" \
 "r4_nolab_a1:200:MI355X_DP_NOL=0 python bench.py --steps 20 --warmup 5" \
 "r4_nolab_b1:200:python bench.py --steps 20 --warmup 5"
