# A/B: non-temporal C stores in the conv / GEMM epilogues (MI_CONV_NTSTORE=1 build variant)
bash tools/gpu_steps.sh \
  nts_r50_base 120 "python bench.py --steps 20 --warmup 5" \
  nts_r50 120 "MI355X_DP_KERNEL_VARIANT=nts python bench.py --steps 20 --warmup 5" \
  nts_vit_base 150 "python bench.py --model vit_b_16 --steps 10 --warmup 3" \
  nts_vit 150 "MI355X_DP_KERNEL_VARIANT=nts python bench.py --model vit_b_16 --steps 10 --warmup 3" \
  nts_r50_base2 120 "python bench.py --steps 20 --warmup 5" \
  nts_r50_2 120 "MI355X_DP_KERNEL_VARIANT=nts python bench.py --steps 20 --warmup 5"
