#!/usr/bin/env python
"""Reference point: the same ResNet training step through STOCK PyTorch-ROCm ops
(MIOpen convs / BN, rocBLAS fc, ATen elementwise, torch.optim.SGD foreach) in
bf16 channels_last.  This is what "PyTorch on MI355X" gives without this
framework's kernels; bench.py is measured against it in profiles/.

    python tools/torch_baseline.py --model resnet50 --batch 256 --steps 20
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn as nn
import torch.nn.functional as F


from mi355x_dp.models.stock import stock_resnet as stock_model  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="resnet50")
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--dtype", default="bf16")
    a = p.parse_args()
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    m = stock_model(a.model, 1000).cuda().to(dt).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(a.batch, 3, a.image_size, a.image_size, device="cuda", dtype=dt).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device="cuda")

    def step():
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        opt.step()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    dt_s = time.perf_counter() - t0
    print(json.dumps({"what": "stock torch eager baseline", "model": a.model, "dtype": a.dtype, "batch": a.batch,
                      "images_per_s": round(a.batch * a.steps / dt_s, 1),
                      "ms_per_step": round(1000 * dt_s / a.steps, 2)}))


if __name__ == "__main__":
    main()
