#!/usr/bin/env python
"""Shadow-model generation time (MNTD C71-C73): K MNIST CNNs trained one after another (the
reference's loop, utils_basic.py:94-117) vs together in one vmapped step (mntd.batched).
Synthetic MNIST-shaped data, 2% shadow split of 60k = 1200 images per model, batch 100, Adam.

    python tools/bench_mntd_train.py [--device cuda] [--models 24] [--epochs 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--models", type=int, default=24)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--n", type=int, default=1200)
    a = ap.parse_args()
    from mi355x_dp.mntd.batched import train_models_batched
    from mi355x_dp.mntd.models import MNISTCNN
    from mi355x_dp.mntd.train import train_model
    dev = torch.device(a.device)
    torch.manual_seed(0)
    # host-resident data, as the reference's loaders (the models move each batch to their device)
    data = [(torch.rand(a.n, 1, 28, 28), torch.randint(0, 10, (a.n,))) for _ in range(a.models)]

    def loaders():
        return [torch.utils.data.DataLoader(torch.utils.data.TensorDataset(*d), batch_size=100, shuffle=True,
                                            generator=torch.Generator(device="cpu").manual_seed(i))
                for i, d in enumerate(data)]

    def models():
        out = []
        for i in range(a.models):
            torch.manual_seed(100 + i)
            out.append(MNISTCNN().to(dev))
        return out

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
    res = {}
    for mode in ("serial", "batched", "serial", "batched"):  # second round: warm
        ms, ls = models(), loaders()
        sync()
        t0 = time.perf_counter()
        if mode == "serial":
            for m, l in zip(ms, ls):
                train_model(m, l, a.epochs, False, verbose=False)
        else:
            train_models_batched(ms, ls, a.epochs, False)
        sync()
        res[mode] = round(time.perf_counter() - t0, 3)
    print(json.dumps({"device": str(dev), "models": a.models, "epochs": a.epochs, "images_per_model": a.n,
                      "serial_s": res["serial"], "batched_s": res["batched"],
                      "speedup": round(res["serial"] / res["batched"], 2)}), flush=True)


if __name__ == "__main__":
    main()
