#!/usr/bin/env python
"""Gradient-precision diagnostic: native bf16 path vs stock-PyTorch bf16 path, both
measured against an fp32 PyTorch reference of the same ResNet weights/batch.
Prints per-parameter relative errors so precision loss can be told from bugs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F


def rel(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12))


def main(model="resnet18", batch=8, size=64, classes=10):
    from mi355x_dp.models import get_model
    from mi355x_dp.ops import cross_entropy
    from mi355x_dp.models.stock import stock_resnet as stock_model

    torch.manual_seed(0)
    m = get_model(model, num_classes=classes).cuda()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(batch, 3, size, size, device="cuda")
    y = torch.randint(0, classes, (batch,), device="cuda")
    cross_entropy(m(x), y).backward()

    ref = stock_model(model, classes).cuda()
    ref.load_state_dict(sd)
    F.cross_entropy(ref(x), y).backward()

    st = stock_model(model, classes).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    st.load_state_dict(sd)
    F.cross_entropy(st(x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)).float(), y).backward()

    names = [n for n, _ in ref.named_parameters()]
    pn = dict(m.named_parameters())
    ps = dict(st.named_parameters())
    pr = dict(ref.named_parameters())
    print(f"{'param':40s} {'native':>9s} {'stock-bf16':>10s}")
    for n in names:
        print(f"{n:40s} {rel(pn[n].grad, pr[n].grad):9.4f} {rel(ps[n].grad, pr[n].grad):10.4f}")


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["resnet18"]))
