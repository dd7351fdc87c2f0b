# end-of-round evidence: RN50 steady-state profile (summary / per-grid / per-launch sequence), ViT
# profile, the smoke entry point, and headline benches
bash tools/gpu_steps_safe.sh \
 "r4_final_smoke:200:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r4_final_prof:400:bash tools/r4_prof_grid.sh r4_final" &&
bash tools/gpu_calls/r4_call29.sh &&
bash tools/gpu_steps_safe.sh \
 "r4_final_rn50_a:200:python bench.py" \
 "r4_final_rn50_b:200:python bench.py --steps 30 --warmup 5" \
 "r4_final_vit:300:python bench.py --model vit_b_16 --steps 10 --warmup 3" \
 "r4_final_rn152:300:python bench.py --model resnet152 --steps 10 --warmup 3"
