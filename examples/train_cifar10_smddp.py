#!/usr/bin/env python
"""SageMaker-style user training script (the kind notebook 2 launches): plain PyTorch DDP code
written against the public APIs the workshop uses -- `smdistributed.dataparallel` backend,
torchvision CIFAR-10 + ResNet-18, DistributedSampler, rank-0 `model.pth` -- running unmodified on
mi355x_dp through the compat packages (SURVEY.md §7.1 decision 1).  Hyperparameters arrive as
`--key value` CLI args and the data/model locations from the SM_* environment.

    python -m mi355x_dp.launch --nproc 8 --sagemaker examples/train_cifar10_smddp.py --epochs 15
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

import smdistributed.dataparallel.torch.torch_smddp  # noqa: F401  (registers the 'smddp' backend)
import torchvision
import torchvision.transforms as T

log = logging.getLogger(__name__)
log.setLevel(logging.INFO)
log.addHandler(logging.StreamHandler(sys.stdout))

MEAN, STD = (0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)


def loaders(data_dir, batch, test_batch, rank, world):
    tf = T.Compose([T.RandomCrop(32, padding=4), T.RandomHorizontalFlip(), T.ToTensor(), T.Normalize(MEAN, STD)])
    train = torchvision.datasets.CIFAR10(root=data_dir, train=True, download=False, transform=tf)
    test = torchvision.datasets.CIFAR10(root=data_dir, train=False, download=False, transform=tf)
    sampler = torch.utils.data.distributed.DistributedSampler(train, num_replicas=world, rank=rank)
    tl = torch.utils.data.DataLoader(train, batch_size=batch, shuffle=False, sampler=sampler, num_workers=0)
    vl = torch.utils.data.DataLoader(test, batch_size=test_batch, shuffle=False, num_workers=0)
    return tl, vl, sampler


def evaluate(model, loader, device):
    model.eval()
    loss, correct = 0.0, 0
    with torch.no_grad():
        for x, y in loader:
            x, y = x.to(device), y.to(device)
            out = model(x).float()
            loss += F.cross_entropy(out, y, reduction="sum").item()
            correct += (out.argmax(1) == y).sum().item()
    n = len(loader.dataset)
    log.info(f"Test set: Average loss: {loss / n:.4f}, Accuracy: {correct / n:.2f}\n")
    return correct / n


def main(args):
    dist.init_process_group(backend=args.backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    device = torch.device("cuda", local_rank) if torch.cuda.is_available() else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    log.info(f"Initialized the distributed environment: '{args.backend}' backend on {world} nodes. "
             f"Current host rank is {rank}. Number of gpus: {args.num_gpus}")
    torch.manual_seed(args.seed)
    per_rank = max(1, args.batch_size // world)  # global batch split over ranks
    tl, vl, sampler = loaders(args.data_dir, per_rank, args.test_batch_size, rank, world)
    model = torchvision.models.resnet18(num_classes=1000).to(device)
    model = torch.nn.parallel.DistributedDataParallel(model)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=args.momentum)
    for epoch in range(1, args.epochs + 1):
        model.train()
        sampler.set_epoch(epoch)
        for i, (x, y) in enumerate(tl):
            x, y = x.to(device), y.to(device)
            opt.zero_grad()
            loss = F.cross_entropy(model(x).float(), y)
            loss.backward()
            opt.step()
            if i % args.log_interval == 0 and rank == 0:
                log.info(f"Train Epoch: {epoch} [{i * len(x)}/{len(sampler)} ({100.0 * i / len(tl):.0f}%)] "
                         f"Loss: {loss.item():.6f}")
        evaluate(model, vl, device)
    if rank == 0:
        log.info("Saving trained model only on rank 0")
        os.makedirs(args.model_dir, exist_ok=True)
        torch.save(model.cpu().state_dict(), os.path.join(args.model_dir, "model.pth"))
    dist.destroy_process_group()


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch-size", type=int, default=256)
    p.add_argument("--test-batch-size", type=int, default=1000)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--log-interval", type=int, default=100)
    p.add_argument("--backend", type=str, default="smddp")
    p.add_argument("--model-dir", type=str, default=os.environ.get("SM_MODEL_DIR", "model"))
    p.add_argument("--data-dir", type=str, default=os.environ.get("SM_CHANNEL_TRAIN", "data"))
    p.add_argument("--num-gpus", type=int, default=int(os.environ.get("SM_NUM_GPUS", "1")))
    p.add_argument("--hosts", type=str, default=os.environ.get("SM_HOSTS", '["algo-1"]'))
    main(p.parse_args())
