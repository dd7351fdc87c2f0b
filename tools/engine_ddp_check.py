#!/usr/bin/env python
"""GPU check of the engine-backed DDP (DataParallel(foreign_optimizer=True), what the torch_smddp
shim substitutes for torch DDP) against the same native model driven by stock optim.SGD without the
engine: per step, the loss and every parameter's gradient and value (relative L2 difference).

    python tools/engine_ddp_check.py [--steps 4] [--model resnet18] [--batch 32] [--size 32]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--wgrad-stream", type=int, default=1)
    a = ap.parse_args()
    from mi355x_dp.models import get_model
    from mi355x_dp.parallel import DataParallel
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    ref = get_model(a.model, num_classes=10).to(dev)
    mod = copy.deepcopy(ref)
    eng = DataParallel(mod, foreign_optimizer=True, wgrad_stream=bool(a.wgrad_stream))
    o_ref = torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9)
    o_eng = torch.optim.SGD(eng.parameters(), lr=0.01, momentum=0.9)
    crit = torch.nn.CrossEntropyLoss()
    names = [n for n, _ in ref.named_parameters()]
    pr = dict(ref.named_parameters())
    pe = dict(mod.named_parameters())
    g = torch.Generator(device=dev).manual_seed(1)
    worst_all = 0.0
    for step in range(a.steps):
        x = torch.randn(a.batch, 3, a.size, a.size, device=dev, generator=g)
        y = torch.randint(0, 10, (a.batch,), device=dev, generator=g)
        losses = []
        for m, o in ((ref, o_ref), (eng, o_eng)):
            o.zero_grad()
            loss = crit(m(x), y)
            loss.backward()
            losses.append(float(loss))
        torch.cuda.synchronize()
        gerr = sorted(((rel(pe[n].grad, pr[n].grad), n) for n in names), reverse=True)
        o_ref.step()
        o_eng.step()
        torch.cuda.synchronize()
        perr = sorted(((rel(pe[n].detach(), pr[n].detach()), n) for n in names), reverse=True)
        worst_all = max(worst_all, gerr[0][0])
        print(f"step {step}: loss ref {losses[0]:.6f} engine {losses[1]:.6f} | worst grad diffs "
              f"{[(round(e, 5), n) for e, n in gerr[:3]]} | worst param diffs {[(round(e, 6), n) for e, n in perr[:2]]}",
              flush=True)
    print("ENGINE_DDP_CHECK", "ok" if worst_all < 5e-2 else "MISMATCH", round(worst_all, 5))


if __name__ == "__main__":
    main()
