#!/usr/bin/env python
"""Can two ranks share one GPU over RCCL on this image?  Each rank binds cuda:0, all-reduces a tensor of
its rank + 1 and prints the result (expected 3.0).  torchrun --nproc-per-node 2 tools/rccl_dup_probe.py"""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
t = torch.full((1 << 20,), float(rank + 1), device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce -> {t[0].item()} (expect 3.0)", flush=True)
dist.destroy_process_group()
