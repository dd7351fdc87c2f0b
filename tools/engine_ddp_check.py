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


def compare(steps=4, model="resnet18", batch=32, size=32, wgrad_stream=True, verbose=True):
    """-> the worst relative gradient / updated-parameter difference over all steps and parameters
    (0.0: bit-exact)"""
    from mi355x_dp.models import get_model
    from mi355x_dp.parallel import DataParallel
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    ref = get_model(model, num_classes=10).to(dev)
    mod = copy.deepcopy(ref)
    eng = DataParallel(mod, foreign_optimizer=True, wgrad_stream=bool(wgrad_stream))
    o_ref = torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9)
    o_eng = torch.optim.SGD(eng.parameters(), lr=0.01, momentum=0.9)
    crit = torch.nn.CrossEntropyLoss()
    names = [n for n, _ in ref.named_parameters()]
    pr = dict(ref.named_parameters())
    pe = dict(mod.named_parameters())
    g = torch.Generator(device=dev).manual_seed(1)
    worst_all = 0.0
    for step in range(steps):
        x = torch.randn(batch, 3, size, size, device=dev, generator=g)
        y = torch.randint(0, 10, (batch,), device=dev, generator=g)
        losses = []
        for m, o in ((ref, o_ref), (eng, o_eng)):
            o.zero_grad()
            out = m(x)
            if m is eng:  # the compute copies the forward used: refreshed from the fp32 masters?
                torch.cuda.synchronize()
                stale = int((eng.flat.bf16 != eng.flat.data.to(torch.bfloat16)).sum())
            loss = crit(out, y)
            loss.backward()
            losses.append(float(loss.detach()))
        torch.cuda.synchronize()
        assert stale == 0, f"step {step}: {stale} bf16 compute-copy elements not refreshed from the fp32 masters"
        assert not eng._final_cb_pending, "the end-of-backward callback did not run"
        gerr = sorted(((rel(pe[n].grad, pr[n].grad), n) for n in names), reverse=True)
        o_ref.step()
        o_eng.step()
        torch.cuda.synchronize()
        perr = sorted(((rel(pe[n].detach(), pr[n].detach()), n) for n in names), reverse=True)
        worst_all = max(worst_all, gerr[0][0], perr[0][0])
        if verbose:
            print(f"step {step}: loss ref {losses[0]:.6f} engine {losses[1]:.6f} | worst grad diffs "
                  f"{[(round(e, 5), n) for e, n in gerr[:3]]} | worst param diffs "
                  f"{[(round(e, 6), n) for e, n in perr[:2]]}", flush=True)
    return worst_all


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--wgrad-stream", type=int, default=1)
    a = ap.parse_args()
    worst = compare(a.steps, a.model, a.batch, a.size, bool(a.wgrad_stream))
    # the native training path is deterministic (no fp32 atomics in the ResNet kernels): bit-exact
    print("ENGINE_DDP_CHECK", "ok" if worst == 0.0 else "MISMATCH", worst)


if __name__ == "__main__":
    main()
