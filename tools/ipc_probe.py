#!/usr/bin/env python
"""Per-size all-reduce path probe of the native smddp backend on this node: RCCL vs the IPC one-shot
and two-shot kernels (mi355x_dp/parallel/comm_paths.py), run as its own N-rank job so a failure
cannot take the caller down.  Rank 0 prints one JSON line {"ipc_probe": {...}}.

    python -m mi355x_dp.launch --nproc N tools/ipc_probe.py      (bench.py runs it after N > 1 jobs)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    from mi355x_dp.parallel.comm_paths import probe_on_new_group
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local % torch.cuda.device_count())
    dev = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group("nccl", device_id=dev)
    res = probe_on_new_group(device=dev)
    if dist.get_rank() == 0:
        print(json.dumps({"ipc_probe": res}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
