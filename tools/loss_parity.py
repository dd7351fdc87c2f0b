#!/usr/bin/env python
"""Training-trajectory parity: the framework's engine (native bf16 kernels, flat-buffer DP,
fused FlatSGD) vs STOCK PyTorch fp32 (ATen/MIOpen convs, torch.optim.SGD) from the same
initial weights on the same fixed batch, same hyper-parameters as bench.py.

Shows that the loss curve bench.py reports (loss_first_warmup -> loss_last) is the curve
a plain PyTorch fp32 training run produces, i.e. the engine trains, it does not just run.

    python tools/loss_parity.py --model resnet50 --batch 64 --steps 30 --lr 0.1
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def run(model="resnet50", batch=64, size=224, classes=1000, steps=30, lr=0.1, momentum=0.9, wd=1e-4, seed=0):
    from mi355x_dp.models import get_model
    from mi355x_dp.models.stock import stock_resnet
    from mi355x_dp.ops import cross_entropy
    from mi355x_dp.parallel import DataParallel, FlatSGD

    dev = torch.device("cuda", 0)
    torch.manual_seed(seed)
    ours = get_model(model, num_classes=classes).to(dev)
    init = {k: v.detach().clone() for k, v in ours.state_dict().items()}
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    x = torch.randn(batch, 3, size, size, device=dev, generator=g)
    y = torch.randint(0, classes, (batch,), device=dev, generator=g)

    engine = DataParallel(ours)
    opt = FlatSGD(engine, lr=lr, momentum=momentum, weight_decay=wd)
    ours_loss = []
    for _ in range(steps):
        engine.zero_grad()
        loss = cross_entropy(engine(x), y)
        loss.backward()
        opt.step()
        ours_loss.append(float(loss.detach()))

    def stock(bf16):
        ref = stock_resnet(model, classes).to(dev)
        ref.load_state_dict(init)
        xin = x
        if bf16:  # stock PyTorch mixed precision: fp32 weights, bf16 autocast compute, channels_last
            ref = ref.to(memory_format=torch.channels_last)
            xin = x.contiguous(memory_format=torch.channels_last)
        ropt = torch.optim.SGD(ref.parameters(), lr=lr, momentum=momentum, weight_decay=wd)
        out = []
        for _ in range(steps):
            ropt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                loss = F.cross_entropy(ref(xin).float(), y)
            loss.backward()
            ropt.step()
            out.append(float(loss.detach()))
        return out

    return ours_loss, stock(False), stock(True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="resnet50")
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--classes", type=int, default=1000)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--lr", type=float, default=0.1)
    a = p.parse_args()
    ours, ref, ref16 = run(a.model, a.batch, a.image_size, a.classes, a.steps, a.lr)
    print(f"{'step':>4} {'engine bf16':>12} {'stock fp32':>12} {'stock bf16':>12}")
    for i, (o, r, h) in enumerate(zip(ours, ref, ref16)):
        print(f"{i:4d} {o:12.4f} {r:12.4f} {h:12.4f}")
    print(json.dumps({"model": a.model, "batch": a.batch, "lr": a.lr, "engine": ours, "stock_fp32": ref,
                      "stock_bf16_autocast": ref16}))


if __name__ == "__main__":
    main()
