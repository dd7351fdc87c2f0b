#!/usr/bin/env python
"""How far ahead of the GPU the host runs in the ResNet-50 bs256 step, without a profiler: events at the
step start, the backward start and the step end; after a synchronize the host clock and the event clock
share an origin (the first event), so each event's lead = GPU time it completed - host time it was
recorded.  python tools/host_lead_probe.py [--steps 8]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--model", default="resnet50")
    a = ap.parse_args()
    from mi355x_dp.models import get_model
    from mi355x_dp.ops import augment, cross_entropy
    from mi355x_dp.parallel import DataParallel, FlatSGD
    dev = torch.device("cuda:0")
    engine = DataParallel(get_model(a.model, num_classes=1000).to(dev))
    opt = FlatSGD(engine, lr=0.1, momentum=0.9, weight_decay=1e-4)
    B = 256
    images = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 1000, (B,), dtype=torch.int64, device=dev)
    x = torch.empty((B, 8, 224, 224), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    marks = []

    def mark(tag):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        marks.append((tag, time.perf_counter(), e))

    def step(i):
        mark(f"s{i} start")
        augment(images, 8, mean, std, pad=0, flip=True, seed=i, out=x)
        engine.zero_grad()
        loss = cross_entropy(engine(x), labels)
        mark(f"s{i} bwd")
        loss.backward()
        mark(f"s{i} opt")
        opt.step()
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    marks.clear()
    mark("origin")
    torch.cuda.synchronize()
    h0, e0 = marks[0][1], marks[0][2]
    for i in range(a.steps):
        step(10 + i)
    mark("end")
    torch.cuda.synchronize()
    print("| event | host ms | GPU ms | lead ms (GPU - host) |\n|---|---:|---:|---:|")
    for tag, h, e in marks[1:]:
        g = e0.elapsed_time(e)
        print(f"| {tag} | {(h - h0) * 1e3:.2f} | {g:.2f} | {g - (h - h0) * 1e3:.2f} |")


if __name__ == "__main__":
    main()
