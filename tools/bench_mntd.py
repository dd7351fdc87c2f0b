#!/usr/bin/env python
"""Meta-classifier epoch time (MNTD, SURVEY.md §3.5: ~0.19 s per 32-model meta-epoch on the
reference's CPU path, dominated by a torch.load per model per step).

Synthetic shadow models of the shipped MNIST CNN shape (random weights; timing does not depend on
the values) are held in a resident ``CheckpointBank``; one epoch = ``epoch_meta_train`` over 32
models (per-model optimizer steps, as the reference) + ``epoch_meta_eval`` over 16 (one vmapped
forward when batched).

    python tools/bench_mntd.py [--device cuda] [--epochs 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--epochs", type=int, default=5)
    a = ap.parse_args()
    import mi355x_dp.mntd.meta as M
    from mi355x_dp.mntd import MNISTCNN
    dev = torch.device(a.device)
    torch.manual_seed(0)
    np.random.seed(0)
    bank = M.CheckpointBank([])
    bank.device = dev
    train, val = [], []
    for i in range(48):
        name = f"synthetic_{i}"
        bank.params[name] = {k: v.to(dev) for k, v in MNISTCNN().state_dict().items()}
        (train if i < 32 else val).append((name, i % 2))
    shadow = MNISTCNN().to(dev)
    res = {"device": str(dev)}
    for batched in (False, True):
        M.BATCHED_EVAL = batched
        meta = M.MetaClassifier((1, 28, 28), 10).to(dev)
        opt = torch.optim.Adam(meta.parameters(), lr=1e-3)
        times = []
        for e in range(a.epochs + 1):
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            M.epoch_meta_train(meta, shadow, opt, train, False, threshold="half", bank=bank)
            M.epoch_meta_eval(meta, shadow, val, False, threshold="half", bank=bank)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            if e:  # first epoch warms up
                times.append(time.perf_counter() - t0)
        t_eval = []
        for _ in range(5):
            t0 = time.perf_counter()
            M.epoch_meta_eval(meta, shadow, val, False, threshold="half", bank=bank)
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t_eval.append(time.perf_counter() - t0)
        key = "batched_eval" if batched else "sequential_eval"
        res[key] = {"meta_epoch_s": round(float(np.median(times)), 4),
                    "eval_16_models_ms": round(1e3 * float(np.median(t_eval)), 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
