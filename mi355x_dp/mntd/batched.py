"""Batched shadow-model training: K same-architecture models trained in ONE vmapped step.

The reference trains its MNTD shadow / target models one after another on the CPU
(train_basic_{benign,jumbo,trojaned}_cpu.py -> utils_basic.py:94-117): tiny
CNNs whose per-model steps are launch-bound on a GPU.  Here the K models' parameters are stacked
(``torch.func.stack_module_state``) and every training step is one ``vmap(grad(loss))`` over the
model axis -- one launch sequence for all K models -- followed by a stacked Adam update with
exactly ``torch.optim.Adam``'s arithmetic (defaults: lr 1e-3, betas (0.9, 0.999), eps 1e-8) and
a per-model step count.

Each model keeps its own DataLoader (own dataset, own shuffle generator).  Models whose loaders
yield batches of different sizes at a step (datasets of different length: jumbo / trojaned
poisoning ratios) are grouped by batch size within the step; a model whose loader is exhausted
simply stops updating until the next epoch.  Dropout draws independent masks per model
(``randomness="different"``).
"""
from __future__ import annotations

import copy
import math
from typing import List, Sequence

import torch
from torch.func import functional_call, grad, stack_module_state, vmap


def train_models_batched(models: Sequence[torch.nn.Module], loaders: Sequence, epoch_num: Sequence[int] | int,
                         is_binary: bool, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                         verbose: bool = False) -> List[torch.nn.Module]:
    """Train ``models`` (same class) on their ``loaders`` for ``epoch_num`` epochs each (an int
    or one per model), in place; returns the models."""
    K = len(models)
    if K == 0:
        return []
    epochs = [epoch_num] * K if isinstance(epoch_num, int) else list(epoch_num)
    for m in models:
        m.train()
    if any(isinstance(mod, torch.nn.RNNBase) for mod in models[0].modules()):
        raise NotImplementedError("train_models_batched: recurrent models (no vmap batching rule for fused RNNs); "
                                  "train them one at a time")
    base = copy.deepcopy(models[0])
    params, buffers = stack_module_state(list(models))
    trainable = {k for k, p in models[0].named_parameters() if p.requires_grad}
    # frozen parameters (the rtNLP model's embedding) ride with the buffers: never differentiated
    buffers = {**{k: v.detach().clone() for k, v in buffers.items()},
               **{k: v.detach().clone() for k, v in params.items() if k not in trainable}}
    params = {k: v.detach().clone() for k, v in params.items() if k in trainable}
    exp_avg = {k: torch.zeros_like(v) for k, v in params.items()}
    exp_avg_sq = {k: torch.zeros_like(v) for k, v in params.items()}
    dev = next(iter(params.values())).device
    steps = torch.zeros(K, dtype=torch.float64)
    b1, b2 = betas

    def loss_fn(p, b, x, y):
        pred = functional_call(base, (p, b), (x,))
        return base.loss(pred, y), pred

    step_fn = vmap(grad(loss_fn, has_aux=True), randomness="different")

    def update(idx: List[int], x, y):
        sel = torch.tensor(idx, device=dev)
        full = len(idx) == K
        p_sub = params if full else {k: v.index_select(0, sel) for k, v in params.items()}
        b_sub = buffers if full else {k: v.index_select(0, sel) for k, v in buffers.items()}
        grads, _ = step_fn(p_sub, b_sub, x, y)
        steps[idx] += 1
        t = steps[idx]
        # torch.optim.Adam: step_size = lr / (1 - b1^t) and sqrt(1 - b2^t) in double, used as fp32
        step = (lr / (1 - b1 ** t)).to(torch.float32).to(dev)
        bc2s = torch.sqrt(1 - b2 ** t).to(torch.float32).to(dev)
        for k, g in grads.items():
            shape = (len(idx),) + (1,) * (g.dim() - 1)
            m = exp_avg[k] if full else exp_avg[k].index_select(0, sel)
            v = exp_avg_sq[k] if full else exp_avg_sq[k].index_select(0, sel)
            p = params[k] if full else params[k].index_select(0, sel)
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v.sqrt() / bc2s.view(shape)).add_(eps)
            p.sub_((m / denom) * step.view(shape))  # = p.addcdiv_(m, denom, value=-step_size)
            if not full:
                exp_avg[k].index_copy_(0, sel, m)
                exp_avg_sq[k].index_copy_(0, sel, v)
                params[k].index_copy_(0, sel, p)

    for epoch in range(max(epochs)):
        iters = [iter(l) if epoch < epochs[i] else None for i, l in enumerate(loaders)]
        while True:
            batch = {}
            for i, it in enumerate(iters):
                if it is None:
                    continue
                try:
                    batch[i] = next(it)
                except StopIteration:
                    iters[i] = None
            if not batch:
                break
            by_size = {}
            for i, (x, y) in batch.items():
                by_size.setdefault(x.shape[0], []).append(i)
            for _, idx in sorted(by_size.items()):
                x = torch.stack([batch[i][0] for i in idx]).to(dev)
                y = torch.stack([batch[i][1] for i in idx]).to(dev)
                update(idx, x, y)
        if verbose:
            print("Epoch %d (batched x%d)" % (epoch, K), flush=True)
    with torch.no_grad():
        for i, m in enumerate(models):
            for k, p in m.named_parameters():
                if k in params:
                    p.copy_(params[k][i])
            for k, b in m.named_buffers():
                if k in buffers:
                    b.copy_(buffers[k][i])
    return list(models)
