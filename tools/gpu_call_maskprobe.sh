# timing probe: what would skipping the dgrad epilogue's BN-output (relu mask) read save?
# (MI_MASK_PROBE=1 variant: mask from the BN input's sign -- wrong results, timing only)
bash tools/gpu_steps.sh \
  mp_base_a 120 "python bench.py --steps 30 --warmup 5" \
  mp_probe_a 120 "MI355X_DP_KERNEL_VARIANT=mprobe python bench.py --steps 30 --warmup 5" \
  mp_base_b 120 "python bench.py --steps 30 --warmup 5" \
  mp_probe_b 120 "MI355X_DP_KERNEL_VARIANT=mprobe python bench.py --steps 30 --warmup 5"
