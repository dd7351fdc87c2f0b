# hypothesis: with a process group the wgrad side stream / comm stream share one of the 4 HW queues
bash tools/gpu_steps.sh \
  hwq_nccl_8 150 "GPU_MAX_HW_QUEUES=8 python bench.py --steps 20 --warmup 5 --force-comm" \
  hwq_plain_8 150 "GPU_MAX_HW_QUEUES=8 python bench.py --steps 20 --warmup 5" \
  hwq_nccl_6 150 "GPU_MAX_HW_QUEUES=6 python bench.py --steps 20 --warmup 5 --force-comm" \
  hwq_nccl_4 150 "python bench.py --steps 20 --warmup 5 --force-comm" \
  hwq_smddp_8 150 "GPU_MAX_HW_QUEUES=8 python bench.py --steps 20 --warmup 5 --force-comm --backend smddp" \
  hwq_plain_4 150 "python bench.py --steps 20 --warmup 5"
