#!/usr/bin/env python
"""PyTorch-side synchronising operations inside a steady-state ResNet-50 bs256 step (torch.cuda sync debug
mode, with the Python stack of each): run two warm-up steps, then two steps with the mode on."""
import os
import sys
import traceback
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from mi355x_dp.models import get_model
    from mi355x_dp.ops import augment, cross_entropy
    from mi355x_dp.parallel import DataParallel, FlatSGD
    dev = torch.device("cuda:0")
    model = get_model("resnet50", num_classes=1000).to(dev)
    engine = DataParallel(model)
    opt = FlatSGD(engine, lr=0.1, momentum=0.9, weight_decay=1e-4)
    B = 256
    images = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 1000, (B,), dtype=torch.int64, device=dev)
    x = torch.empty((B, 8, 224, 224), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)

    def step(i):
        augment(images, 8, mean, std, pad=0, flip=True, seed=i, out=x)
        engine.zero_grad()
        loss = cross_entropy(engine(x), labels)
        loss.backward()
        opt.step()

    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    seen = {}

    def show(message, category, filename, lineno, file=None, line=None):
        stack = "".join(traceback.format_stack(limit=12)[:-1])
        key = stack
        seen[key] = seen.get(key, 0) + 1
        if seen[key] == 1:
            print(f"--- {message}\n{stack}", flush=True)
    warnings.showwarning = show
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    for i in range(2):
        step(10 + i)
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    print(f"distinct synchronising call sites in 2 steps: {len(seen)}; total hits {sum(seen.values())}")


if __name__ == "__main__":
    main()
