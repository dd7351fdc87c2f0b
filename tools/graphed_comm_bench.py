#!/usr/bin/env python
"""ms/step of the reference loop shape (ResNet-18, 1000 classes, batch 32 at 32x32, stock SGD through
the engine-backed DDP, graphed steps) at world 1 with every bucket collective issued
(MI355X_DP_FORCE_COMM=1) -- collectives captured into the backward graph, behind per-bucket gates
enqueued before the replay, or all launched after the replay -- and without collectives.  One
process, so it can run under rocprofv3.

    python tools/graphed_comm_bench.py --mode capture|gated|ungated|nocomm [--backend smddp|nccl] [--steps 300]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.append(os.path.join(ROOT, "compat"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="capture", choices=("capture", "gated", "ungated", "nocomm"))
    p.add_argument("--backend", default="smddp")
    p.add_argument("--steps", type=int, default=300)
    a = p.parse_args()
    os.environ["MI355X_DP_FORCE_COMM"] = "0" if a.mode == "nocomm" else "1"
    os.environ["MI355X_DP_GRAPH_COMM"] = {"capture": "capture", "gated": "gates", "ungated": "after",
                                          "nocomm": "auto"}[a.mode]
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29577")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("LOCAL_RANK", "0")
    from mi355x_dp.utils import hwqueues
    hwqueues.ensure()
    import torch
    import torch.distributed as dist
    import smdistributed.dataparallel.torch.torch_smddp  # noqa: F401
    dist.init_process_group(backend=a.backend)
    torch.cuda.set_device(0)
    from mi355x_dp.models import get_model
    torch.manual_seed(0)
    ddp = torch.nn.parallel.DistributedDataParallel(get_model("resnet18", num_classes=1000).cuda())
    opt = torch.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9)
    crit = torch.nn.CrossEntropyLoss().cuda()
    x = torch.randn(32, 3, 32, 32, device="cuda")
    y = torch.randint(0, 1000, (32,), device="cuda")

    host = {"gated_launch": 0.0, "finish": 0.0, "replay": 0.0}
    eng = ddp
    if hasattr(eng, "_gated_launch"):
        orig_gl, orig_fin = eng._gated_launch, eng.finish_gradient_sync

        def gl(*args, **kw):
            t = time.perf_counter()
            r = orig_gl(*args, **kw)
            host["gated_launch"] += time.perf_counter() - t
            return r

        def fin(*args, **kw):
            t = time.perf_counter()
            r = orig_fin(*args, **kw)
            host["finish"] += time.perf_counter() - t
            return r
        eng._gated_launch, eng.finish_gradient_sync = gl, fin

    ph = {"zero": 0.0, "fwd": 0.0, "bwd": 0.0, "opt": 0.0}

    def step():
        t = time.perf_counter()
        opt.zero_grad()
        t1 = time.perf_counter()
        loss = crit(ddp(x), y)
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        opt.step()
        t4 = time.perf_counter()
        ph["zero"] += t1 - t
        ph["fwd"] += t2 - t1
        ph["bwd"] += t3 - t2
        ph["opt"] += t4 - t3
        return loss
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    ms = 1000 * (time.perf_counter() - t0) / a.steps
    host = {k: round(1000 * v / (a.steps + 10), 4) for k, v in list(host.items()) + list(ph.items())}
    modes = sorted({s.comm_mode for s in getattr(ddp, "_graphs", {}).values()})
    print(json.dumps({"mode": a.mode, "backend": a.backend, "ms_per_step": round(ms, 4), "comm_modes": modes,
                      "img_s": round(32 / ms * 1000, 1), "loss": float(loss), "host_ms": host}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
