bash tools/gpu_steps_safe.sh \
 "r4_gpu_full3:1000:python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread" &&
bash tools/gpu_steps_safe.sh \
 "r4_smoke3:200:python -c 'import __graft_entry__ as g; g.smoke()'"
