"""Basic trainer / evaluator for MNTD target models (reference utils_basic.py:94-134, C70)
and the shadow/target model generation drivers (train_basic_{benign,jumbo,trojaned}_cpu.py,
C71-C73), plus their distributed form (C74).

The reference's "distributed" variants do not parse (TabError) and would not run
(DDP(device_ids=[rank]) on CPU models, ``model.loss`` on the DDP wrapper, undefined
``args.troj_type``, nccl with CPU tensors).  The natural MI355X design
is implemented instead: *task parallelism* -- rank r of W trains shadow models
r, r+W, r+2W, ... on its own GPU (or CPU), with the same per-model seeds as the
serial run, and rank 0 gathers the accuracies into the JSON log.
"""
from __future__ import annotations

import argparse
import json
import os
from datetime import datetime

import numpy as np
import torch
import torch.utils.data

from .data import BackdoorDataset, load_dataset_setting


def train_model(model, dataloader, epoch_num, is_binary, verbose=True):
    model.train()
    optimizer = torch.optim.Adam(model.parameters(), lr=1e-3)
    for epoch in range(epoch_num):
        cum_loss = cum_acc = tot = 0.0
        for x_in, y_in in dataloader:
            B = x_in.size(0)
            pred = model(x_in)
            loss = model.loss(pred, y_in)
            optimizer.zero_grad()
            loss.backward()
            optimizer.step()
            cum_loss += loss.item() * B
            if is_binary:
                cum_acc += ((pred > 0).cpu().long().eq(y_in)).sum().item()
            else:
                cum_acc += (pred.max(1)[1].cpu().eq(y_in)).sum().item()
            tot += B
        if verbose:
            print("Epoch %d, loss = %.4f, acc = %.4f" % (epoch, cum_loss / tot, cum_acc / tot))


@torch.no_grad()
def eval_model(model, dataloader, is_binary):
    model.eval()
    cum_acc = tot = 0.0
    for x_in, y_in in dataloader:
        pred = model(x_in)
        if is_binary:
            cum_acc += ((pred > 0).cpu().long().eq(y_in)).sum().item()
        else:
            cum_acc += (pred.max(1)[1].cpu().eq(y_in)).sum().item()
        tot += x_in.size(0)
    return cum_acc / tot


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def generate(task, kind, troj_type="M", shadow_prop=0.02, target_prop=0.5, shadow_num=24, target_num=8,
             n_epoch=None, gpu=False, save_root="./shadow_model_ckpt", data_root="./raw_data/", verbose=False,
             limit_train=None, batched=False):
    """kind: 'benign' (shadow_benign_i + target_benign_i), 'jumbo' (shadow_jumbo_i),
    'trojaned' (target_troj{M,B}_i).  Returns the JSON log dict (written by rank 0).
    ``batched=True``: this rank's models train together, one vmapped step for all of them
    (``mntd.batched``) -- same initial weights, same per-model data order, same Adam arithmetic as
    the one-at-a-time loop."""
    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    np.random.seed(0)
    torch.manual_seed(0)
    bs, ne, trainset, testset, is_binary, need_pad, Model, troj_gen, troj_setting = load_dataset_setting(
        task, data_root)
    if limit_train:
        trainset = torch.utils.data.Subset(trainset, range(min(limit_train, len(trainset))))
    n_epoch = n_epoch or ne
    tot = len(trainset)
    shadow_idx = np.random.choice(tot, int(tot * shadow_prop))
    target_idx = np.random.choice(tot, int(tot * target_prop))
    save_dir = os.path.join(save_root, task, "models")
    if rank == 0:
        os.makedirs(save_dir, exist_ok=True)
    if dist:
        dist.barrier()
    testloader = torch.utils.data.DataLoader(testset, batch_size=bs)
    jobs = []
    if kind == "benign":
        jobs = [("shadow_benign_%d" % i, shadow_idx, n_epoch, None) for i in range(shadow_num)]
        jobs += [("target_benign_%d" % i, target_idx, max(1, int(n_epoch * shadow_prop / target_prop)), None)
                 for i in range(target_num)]
    elif kind == "jumbo":
        jobs = [("shadow_jumbo_%d" % i, shadow_idx, n_epoch, "jumbo") for i in range(shadow_num)]
    elif kind == "trojaned":
        jobs = [("target_troj%s_%d" % (troj_type, i), target_idx, max(1, int(n_epoch * shadow_prop / target_prop)),
                 troj_type) for i in range(target_num)]
    else:
        raise ValueError(kind)
    # attack settings drawn serially (same RNG stream as the single-process reference run)
    settings = [troj_setting(t) if t else None for (_, _, _, t) in jobs]
    results = {}
    mine = []
    for j, ((name, idx, ep, t), atk) in enumerate(zip(jobs, settings)):
        if j % world != rank:
            continue
        torch.manual_seed(1000 + j)  # per-model seeds: identical models whichever rank trains them
        np.random.seed(1000 + j)
        model = Model(gpu=gpu)
        # per-model shuffle generator: the data order does not depend on which rank trains the
        # model or whether it trains alone or batched with others
        shuf = torch.Generator().manual_seed(2000 + j)
        if atk is None:
            loader = torch.utils.data.DataLoader(torch.utils.data.Subset(trainset, idx), batch_size=bs, shuffle=True,
                                                 generator=shuf)
        else:
            loader = torch.utils.data.DataLoader(BackdoorDataset(trainset, atk, troj_gen, choice=idx,
                                                                 need_pad=need_pad), batch_size=bs, shuffle=True,
                                                 generator=shuf)
        mine.append((name, model, loader, ep, atk))
    if batched and mine and any(isinstance(mod, torch.nn.RNNBase) for mod in mine[0][1].modules()):
        print("batched training: recurrent model (%s), training one model at a time" % type(mine[0][1]).__name__)
        batched = False
    if batched and mine:
        from .batched import train_models_batched
        train_models_batched([m for _, m, _, _, _ in mine], [l for _, _, l, _, _ in mine], [e for *_, e, _ in mine],
                             is_binary, verbose=verbose)
    for name, model, loader, ep, atk in mine:
        if not batched:
            train_model(model, loader, ep, is_binary, verbose=verbose)
        path = os.path.join(save_dir, name + ".model")
        torch.save(model.state_dict(), path)
        acc = eval_model(model, testloader, is_binary)
        line = "Acc %.4f, " % acc
        acc_mal = None
        if atk is not None:
            mal = torch.utils.data.DataLoader(BackdoorDataset(testset, atk, troj_gen, mal_only=True), batch_size=bs)
            acc_mal = eval_model(model, mal, is_binary)
            line += "Acc on backdoor %.4f, " % acc_mal
        print(line + "saved to %s @ %s" % (path, datetime.now()), flush=True)
        results[name] = (acc, acc_mal)
    if dist:
        gathered = [None] * world
        dist.all_gather_object(gathered, results)
        results = {k: v for d in gathered for k, v in d.items()}
    accs = [a for a, _ in results.values()]
    mals = [m for _, m in results.values() if m is not None]
    log = {"kind": kind, "task": task, "n_models": len(results), "acc": float(np.mean(accs)) if accs else None}
    if mals:
        log["acc_mal"] = float(np.mean(mals))
    if rank == 0:
        name = {"benign": "benign", "jumbo": "jumbo", "trojaned": "troj%s" % troj_type}[kind]
        with open(os.path.join(save_root, task, name + ".log"), "w") as f:
            json.dump(log, f)
    return log


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m mi355x_dp.mntd.train")
    ap.add_argument("--task", required=True)
    ap.add_argument("--kind", choices=["benign", "jumbo", "trojaned"], required=True)
    ap.add_argument("--troj_type", default="M")
    ap.add_argument("--epochs", type=int, default=None)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--distributed", action="store_true", help="task-parallel over WORLD_SIZE ranks (gloo/smddp)")
    ap.add_argument("--batched", action="store_true", help="train this rank's models together (one vmapped step)")
    a = ap.parse_args(argv)
    if a.distributed:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    print(json.dumps(generate(a.task, a.kind, a.troj_type, n_epoch=a.epochs, gpu=a.gpu, batched=a.batched)))


if __name__ == "__main__":
    main()
