B="python bench.py --steps 30 --warmup 5"
bash tools/gpu_steps.sh \
  mp_base 120 "$B" \
  mp_hi 120 "MI355X_DP_MAIN_PRIORITY=-1 $B" \
  mp_base2 120 "$B" \
  mp_hi2 120 "MI355X_DP_MAIN_PRIORITY=-1 $B" \
  mp_hi_force 120 "MI355X_DP_MAIN_PRIORITY=-1 $B --force-comm" \
  mp_force 120 "$B --force-comm"
