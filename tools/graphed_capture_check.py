#!/usr/bin/env python
"""The graphed engine's three ways of issuing a replayed backward's bucket collectives
(parallel/step_graph.py ``comm_mode``: ``capture`` -- captured into the backward graph, ``gates`` --
gate kernels + collectives enqueued before the replay, ``after`` -- all launched after it) against
the eager engine, at world 1 with every collective issued (force_comm), on one backend.  Runs the
reference loop shape (ResNet-18, 1000-class head, batch 32 at 32x32, stock SGD, a short batch and an
eval pass in between) and prints one JSON line: per-mode losses, whether every mode's final flat
fp32 parameters and BN buffers equal the eager run's bit for bit, the comm modes the captured steps
used, replays, and the number of collectives issued.

    python tools/graphed_capture_check.py --backend nccl|smddp
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.append(os.path.join(ROOT, "compat"))


def run(graph, comm, steps=9):
    import torch
    from mi355x_dp.models import get_model
    from mi355x_dp.parallel import DataParallel, step_graph
    step_graph.MODE = graph
    step_graph.GRAPH_COMM = comm
    torch.manual_seed(0)
    eng = DataParallel(get_model("resnet18", num_classes=1000).cuda(), foreign_optimizer=True, wgrad_stream=False,
                       force_comm=True)
    opt = torch.optim.SGD(eng.parameters(), lr=0.01, momentum=0.9)
    crit = torch.nn.CrossEntropyLoss().cuda()
    g = torch.Generator().manual_seed(5)
    losses = []
    for i in range(steps):
        n = 32 if i != steps - 2 else 10
        data = torch.randn(n, 3, 32, 32, generator=g).cuda()
        target = torch.randint(0, 10, (n,), generator=g).cuda()
        opt.zero_grad()
        loss = crit(eng(data), target)
        loss.backward()
        opt.step()
        losses.append(float(loss))
        if i == 4:
            eng.eval()
            with torch.no_grad():
                eng(torch.randn(100, 3, 32, 32, generator=g).cuda())
            eng.train()
    torch.cuda.synchronize()
    graphs = getattr(eng, "_graphs", {})
    return {"losses": losses, "flat": eng.flat.data.clone(), "bufs": eng.buffers.data.clone(),
            "modes": sorted({s.comm_mode for s in graphs.values()}),
            "replays": sum(s.replays for s in graphs.values()), "comm_calls": eng.comm_calls}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl")
    a = ap.parse_args()
    for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29591"), ("RANK", "0"), ("WORLD_SIZE", "1"),
                 ("LOCAL_RANK", "0")):
        os.environ.setdefault(k, v)
    from mi355x_dp.utils import hwqueues
    hwqueues.ensure()
    import torch
    import torch.distributed as dist
    import smdistributed.dataparallel.torch.torch_smddp  # noqa: F401  (registers 'smddp')
    torch.cuda.set_device(0)
    dist.init_process_group(backend=a.backend)
    ref = run("0", "auto")
    out = {"backend": a.backend, "eager_losses": ref["losses"], "eager_comm_calls": ref["comm_calls"]}
    for comm in ("capture", "gates", "after"):
        r = run("1", comm)
        out[comm] = {"modes": r["modes"], "replays": r["replays"], "comm_calls": r["comm_calls"],
                     "losses_equal": r["losses"] == ref["losses"],
                     "params_equal": bool(torch.equal(r["flat"], ref["flat"])),
                     "buffers_equal": bool(torch.equal(r["bufs"], ref["bufs"]))}
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
