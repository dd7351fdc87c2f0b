#!/usr/bin/env python
"""All-reduce latency / bus bandwidth per size: torch `nccl` (RCCL over xGMI) vs the native
`smddp` backend (RCCL, or the IPC one-shot / two-shot kernels with MI355X_DP_SMDDP_IPC=1).
Used to pick MI355X_DP_SMDDP_IPC_ONESHOT_KB / MI355X_DP_SMDDP_IPC_MB and the DDP bucket sizes.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py --backend nccl
    MI355X_DP_SMDDP_IPC=1 torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py --backend smddp

Bus bandwidth uses the ring convention 2 (w - 1) / w x bytes / time (as nccl-tests).
Rank 0 prints one JSON line per size (time = mean over ranks).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.append(os.path.join(ROOT, "compat"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl", choices=["nccl", "smddp", "gloo"])
    ap.add_argument("--sizes-kb", default="4,64,256,1024,4096,16384,65536")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", int(os.environ.get("MI355X_DP_SMDDP_DEVICE", local)))
    torch.cuda.set_device(dev)
    if a.backend == "smddp":
        import smdistributed.dataparallel.torch.torch_smddp  # noqa: F401  registers 'smddp'
        dist.init_process_group("smddp")
    else:
        dist.init_process_group(a.backend)
    w, r = dist.get_world_size(), dist.get_rank()
    for kb in [int(x) for x in a.sizes_kb.split(",")]:
        t = torch.ones(kb * 256, device=dev, dtype=torch.float32)
        for _ in range(a.warmup):
            dist.all_reduce(t)
        torch.cuda.synchronize()
        dist.all_reduce(torch.zeros(1, device=dev))  # barrier (fp32 SUM: stays on the IPC path too)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            dist.all_reduce(t)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / a.iters
        mean = torch.tensor([us], device=dev)
        dist.all_reduce(mean)  # rank-mean time (SUM keeps it IPC-eligible)
        us = float(mean) / w
        if r == 0:
            busbw = 2.0 * (w - 1) / w * kb * 1024 / (us * 1e-6) / 1e9
            print(json.dumps({"backend": a.backend, "ipc": os.environ.get("MI355X_DP_SMDDP_IPC", "0"),
                              "world": w, "kb": kb, "us": round(us, 1), "busbw_GBps": round(busbw, 1)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
