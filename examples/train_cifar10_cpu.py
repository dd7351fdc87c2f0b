#!/usr/bin/env python
"""Notebook-1-style user training script: LeNet on CIFAR-10, one process per "host", gloo
DistributedDataParallel on CPU, rank-0 `model.pth` with bare `Net` keys (what a CPU SageMaker job
writes).  Hosts, rank, model and data locations come from the SM_* contract
that mi355x_dp's local job runner sets; hyperparameters arrive as `--key value` CLI args.

    python -m mi355x_dp.launch --nproc 2 --sagemaker examples/train_cifar10_cpu.py --epochs 20
    (or PyTorch(entry_point="train_cifar10_cpu.py", instance_count=2, ...).fit(), notebooks/1_*.ipynb)
"""
import argparse
import json
import logging
import os
import sys

import torch
import torch.distributed as dist
import torch.nn.functional as F
import torch.utils.data
import torch.utils.data.distributed

import torchvision
import torchvision.transforms as T
from mi355x_dp.models.lenet import Net

log = logging.getLogger(__name__)
log.setLevel(logging.INFO)
log.addHandler(logging.StreamHandler(sys.stdout))

MEAN, STD = (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)


def loaders(data_dir, batch, test_batch, rank, world):
    tf = T.Compose([T.RandomCrop(32, padding=4), T.RandomHorizontalFlip(), T.ToTensor(), T.Normalize(MEAN, STD)])
    test_tf = T.Compose([T.ToTensor(), T.Normalize(MEAN, STD)])
    train = torchvision.datasets.CIFAR10(root=data_dir, train=True, download=False, transform=tf)
    test = torchvision.datasets.CIFAR10(root=data_dir, train=False, download=False, transform=test_tf)
    sampler = torch.utils.data.distributed.DistributedSampler(train, num_replicas=world, rank=rank)
    tl = torch.utils.data.DataLoader(train, batch_size=batch, sampler=sampler, num_workers=0)
    vl = torch.utils.data.DataLoader(test, batch_size=test_batch, shuffle=False, num_workers=0)
    return tl, vl, sampler


def evaluate(model, loader):
    model.eval()
    loss, correct = 0.0, 0
    with torch.no_grad():
        for x, y in loader:
            out = model(x)
            loss += F.cross_entropy(out, y, reduction="sum").item()
            correct += (out.argmax(1) == y).sum().item()
    n = len(loader.dataset)
    log.info(f"Test set: Average loss: {loss / n:.4f}, Accuracy: {correct / n:.2f}\n")
    return correct / n


def main(args):
    hosts = json.loads(args.hosts)
    world, rank = len(hosts), hosts.index(args.current_host)
    distributed = world > 1
    if distributed:
        dist.init_process_group(backend=args.backend, rank=rank, world_size=world)
        log.info(f"Initialized the distributed environment: '{args.backend}' backend on {world} nodes. "
                 f"Current host rank is {rank}.")
    torch.manual_seed(args.seed)
    tl, vl, sampler = loaders(args.data_dir, args.batch_size, args.test_batch_size, rank, world)
    model = Net()
    if distributed:
        model = torch.nn.parallel.DistributedDataParallel(model)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=args.momentum)
    for epoch in range(1, args.epochs + 1):
        model.train()
        sampler.set_epoch(epoch)
        for i, (x, y) in enumerate(tl):
            opt.zero_grad()
            loss = F.cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            if i % args.log_interval == 0:
                log.info(f"Train Epoch: {epoch} [{i * len(x)}/{len(sampler)} ({100.0 * i / len(tl):.0f}%)] "
                         f"Loss: {loss.item():.6f}")
        evaluate(model, vl)
    if rank == 0:
        log.info("Saving the model.")
        os.makedirs(args.model_dir, exist_ok=True)
        net = model.module if distributed else model
        torch.save(net.state_dict(), os.path.join(args.model_dir, "model.pth"))  # bare Net keys
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--test-batch-size", type=int, default=1000)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--log-interval", type=int, default=100)
    p.add_argument("--backend", type=str, default="gloo")
    p.add_argument("--model-type", type=str, default="custom")
    p.add_argument("--hosts", type=str, default=os.environ.get("SM_HOSTS", '["algo-1"]'))
    p.add_argument("--current-host", type=str, default=os.environ.get("SM_CURRENT_HOST", "algo-1"))
    p.add_argument("--model-dir", type=str, default=os.environ.get("SM_MODEL_DIR", "model"))
    p.add_argument("--data-dir", type=str, default=os.environ.get("SM_CHANNEL_TRAIN", "data"))
    main(p.parse_args())
