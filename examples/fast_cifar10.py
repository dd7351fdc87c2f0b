#!/usr/bin/env python
"""Reference-parity job on the native engine (BASELINE.md "what we will measure", item 1):
ResNet-18 (torchvision layout, 1000-class head) on CIFAR-10-shaped data, 15 epochs, global
batch 256, SGD(lr 0.01, momentum 0.9) -- the notebook-2 hyperparameters -- but with the dataset
resident in HBM as uint8, the fused augmentation kernel, the flat-buffer DP engine and the
training step replayed as one HIP graph.  Prints the reference's log lines per epoch and a JSON
summary (loop seconds, images/s, final accuracy) to compare with the reference job's
438 s billed / ~166 s training loop / >= 4.5k img/s on 8 x A100.

    python examples/fast_cifar10.py [--data DIR_WITH_cifar-10-batches-py] [--epochs 15]
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/fast_cifar10.py
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MEAN, STD = (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)


def load_data(path, n_train, n_test, seed):
    """uint8 NHWC arrays from the official pickle layout (safe unpickler), or synthetic."""
    import numpy as np
    from mi355x_dp.data.cifar import load_cifar10, write_synthetic_cifar10
    if path is None:
        import tempfile
        path = tempfile.mkdtemp(prefix="cifar_syn_")
        write_synthetic_cifar10(path, n_train=n_train, n_test=n_test, seed=seed)
    xtr, ytr = load_cifar10(path, train=True)
    xte, yte = load_cifar10(path, train=False)
    return np.ascontiguousarray(xtr), np.asarray(ytr), np.ascontiguousarray(xte), np.asarray(yte)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", default=None)
    ap.add_argument("--epochs", type=int, default=15)
    ap.add_argument("--global-batch", type=int, default=256)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--n-train", type=int, default=50000)
    ap.add_argument("--n-test", type=int, default=10000)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    t_job = time.time()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    from mi355x_dp.models import get_model
    from mi355x_dp.ops import augment, cross_entropy
    from mi355x_dp.parallel import DataParallel, FlatSGD

    xtr, ytr, xte, yte = load_data(a.data, a.n_train, a.n_test, a.seed)
    imgs = torch.from_numpy(xtr).to(dev)                 # [N, 32, 32, 3] uint8, resident in HBM
    labels = torch.from_numpy(ytr).long().to(dev)
    timgs = torch.from_numpy(xte).to(dev)
    tlabels = torch.from_numpy(yte).long().to(dev)
    if rank == 0:
        print(f"Initialized the distributed environment: 'nccl' backend on {world} nodes. ", flush=True)
    torch.manual_seed(a.seed)
    engine = DataParallel(get_model("resnet18", num_classes=1000).to(dev))
    opt = FlatSGD(engine, lr=a.lr, momentum=a.momentum)
    B = a.global_batch // world
    shard = torch.arange(rank, imgs.shape[0], world, device=dev)   # DistributedSampler split
    steps = shard.numel() // B                                       # static shapes: drop the last partial batch
    if rank == 0:
        print(f"Processes {shard.numel()}/{imgs.shape[0]} ({100.0 * shard.numel() / imgs.shape[0]:.0f}%) of train data",
              flush=True)

    u8 = torch.empty((B, 32, 32, 3), dtype=torch.uint8, device=dev)
    yb = torch.empty((B,), dtype=torch.long, device=dev)
    x = torch.empty((B, 8, 32, 32), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)

    def core():
        engine.zero_grad()
        loss = cross_entropy(engine(x), yb)
        loss.backward()
        opt.step()
        return loss

    graphed, step_no = None, 0

    def train_step(idx):
        nonlocal graphed, step_no
        torch.index_select(imgs, 0, idx, out=u8)
        torch.index_select(labels, 0, idx, out=yb)
        augment(u8, 8, MEAN, STD, pad=4, flip=True, seed=a.seed * 1000003 + step_no, out=x)
        step_no += 1
        if a.no_graph or step_no == 1:
            return core()
        if graphed is None:
            from mi355x_dp.graphs import GraphedStep
            graphed = GraphedStep(core, warmup=1)
        return graphed()

    def evaluate():
        engine.eval()
        loss, correct = 0.0, 0
        with torch.no_grad():
            for i in range(0, timgs.shape[0], 1000):
                xt = augment(timgs[i:i + 1000], 8, MEAN, STD, pad=4, flip=True, seed=99 + i)
                out = engine(xt).float()
                y = tlabels[i:i + 1000]
                loss += float(torch.nn.functional.nll_loss(out, y, reduction="sum"))  # reference: nll on logits
                correct += int((out.argmax(1) == y).sum())
        engine.train()
        n = timgs.shape[0]
        return loss / n, correct / n

    torch.cuda.synchronize()
    t_loop = time.time()
    train_time = 0.0
    acc = 0.0
    g = torch.Generator(device=dev)
    for epoch in range(1, a.epochs + 1):
        g.manual_seed(a.seed + epoch)
        order = shard[torch.randperm(shard.numel(), device=dev, generator=g)]
        torch.cuda.synchronize()
        t0 = time.time()
        for s in range(steps):
            loss = train_step(order[s * B:(s + 1) * B])
            if s % 100 == 0 and rank == 0:
                print(f"Train Epoch: {epoch} [{s * B}/{shard.numel()} ({100.0 * s / steps:.0f}%)] "
                      f"Loss: {float(loss):.6f}", flush=True)
        torch.cuda.synchronize()
        train_time += time.time() - t0
        tl, acc = evaluate()
        if rank == 0:
            print(f"Test set: Average loss: {tl:.4f}, Accuracy: {acc:.2f}\n", flush=True)
    loop_s = time.time() - t_loop
    if rank == 0:
        imgs_trained = a.epochs * steps * B * world
        print(json.dumps({"job_seconds": round(time.time() - t_job, 2), "loop_seconds": round(loop_s, 2),
                          "train_seconds": round(train_time, 2), "train_images_per_s": round(imgs_trained / train_time),
                          "final_test_accuracy": round(acc, 4), "epochs": a.epochs, "global_batch": a.global_batch,
                          "world_size": world, "hip_graph": not a.no_graph,
                          "data": "synthetic CIFAR-10 layout" if a.data is None else a.data}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
