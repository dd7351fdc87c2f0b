#!/usr/bin/env python
"""GPU check for reads of uninitialised memory in the native training path: every ``torch.empty``
is filled with NaN (``torch.utils.deterministic.fill_uninitialized_memory`` under deterministic
mode), so a kernel that reads a workspace row or output element nobody wrote turns the loss or a
gradient into NaN.  Also repeats the same step twice from identical state and compares the
gradients bitwise (a race or an uninitialised read shows up as a difference).

    python tools/uninit_check.py [--model resnet18] [--batch 32] [--size 32] [--classes 10]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--classes", type=int, default=10)
    ap.add_argument("--nan-fill", type=int, default=1)
    a = ap.parse_args()
    from mi355x_dp.models import get_model
    if a.nan_fill:
        torch.use_deterministic_algorithms(True, warn_only=True)
        torch.utils.deterministic.fill_uninitialized_memory = True
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m0 = get_model(a.model, num_classes=a.classes).to(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(a.batch, 3, a.size, a.size, device=dev, generator=g)
    y = torch.randint(0, a.classes, (a.batch,), device=dev, generator=g)
    crit = torch.nn.CrossEntropyLoss()
    runs = []
    for rep in range(3):
        m = copy.deepcopy(m0)
        loss = crit(m(x), y)
        loss.backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        bufs = {n: b.detach().clone() for n, b in m.named_buffers()}
        bad = [n for n, t in grads.items() if not torch.isfinite(t).all()]
        badb = [n for n, t in bufs.items() if t.is_floating_point() and not torch.isfinite(t).all()]
        print(f"rep {rep}: loss {float(loss.detach()):.6f} non-finite grads {len(bad)} {bad[:6]} "
              f"non-finite buffers {badb[:4]}", flush=True)
        runs.append((float(loss.detach()), grads))
    diffs = []
    for n, t in runs[0][1].items():
        for r in runs[1:]:
            d = (t.double() - r[1][n].double()).abs().max().item()
            if not d == 0.0:
                diffs.append((d, n))
    diffs.sort(reverse=True)
    print(f"repeat differences: {len(diffs)} params differ; worst {diffs[:6]}", flush=True)
    ok = not diffs and all(torch.isfinite(torch.tensor(l)) for l, _ in runs)
    print("UNINIT_CHECK", "ok" if ok else "FAIL")


if __name__ == "__main__":
    main()
