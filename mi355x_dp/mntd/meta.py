"""Meta-classifier and meta-training (reference notebooks/code/meta_classifier.py,
utils_meta.py).

MI355X-first changes to the hot loop (which in the reference is dominated by
``torch.load`` of a ~1.1 MB checkpoint per model per step): a
``CheckpointBank`` loads every shadow/target state_dict ONCE (``weights_only=True``) and
keeps them resident on the device; each step swaps parameters with
``torch.func.functional_call`` (no copies, no file I/O); evaluation runs all models of a split in ONE ``torch.func.vmap``
forward over the bank's stacked parameters (``_eval_scores_batched``).  Semantics -- per-model
forward of the learnable queries, BCE / one-class loss, per-model optimizer step,
AUC via sklearn, 'half' = median threshold -- are unchanged.  ``np.asscalar`` (gone
in numpy 2) is replaced by ``float``.
"""
from __future__ import annotations

import os
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.func import functional_call, stack_module_state, vmap

from .models import TASK_MODELS


class MetaClassifier(nn.Module):
    def __init__(self, input_size, class_num, N_in=10, gpu=False):
        super().__init__()
        self.input_size, self.class_num, self.N_in, self.N_h = input_size, class_num, N_in, 20
        self.inp = nn.Parameter(torch.zeros(self.N_in, *input_size).normal_() * 1e-3)
        self.fc = nn.Linear(self.N_in * self.class_num, self.N_h)
        self.output = nn.Linear(self.N_h, 1)
        self.gpu = gpu
        if gpu and torch.cuda.is_available():
            self.cuda()

    def forward(self, pred):
        emb = F.relu(self.fc(pred.reshape(self.N_in * self.class_num)))
        return self.output(emb)

    def loss(self, score, y):
        return F.binary_cross_entropy_with_logits(score, torch.tensor([float(y)], device=score.device))


class MetaClassifierOC(nn.Module):
    """One-class variant: hinge on radius r, r updated to the v-percentile of scores."""

    def __init__(self, input_size, class_num, N_in=10, gpu=False):
        super().__init__()
        self.N_in, self.N_h, self.v = N_in, 20, 0.1
        self.input_size, self.class_num = input_size, class_num
        self.inp = nn.Parameter(torch.zeros(self.N_in, *input_size).normal_() * 1e-3)
        self.fc = nn.Linear(self.N_in * self.class_num, self.N_h)
        self.w = nn.Parameter(torch.zeros(self.N_h).normal_() * 1e-3)
        self.r = 1.0
        if gpu and torch.cuda.is_available():
            self.cuda()

    def forward(self, pred, ret_feature=False):
        emb = F.relu(self.fc(pred.reshape(self.N_in * self.class_num)))
        return emb if ret_feature else torch.dot(emb, self.w)

    def loss(self, score):
        reg = (self.w ** 2).sum() / 2
        for p in self.fc.parameters():
            reg = reg + (p ** 2).sum() / 2
        return reg + F.relu(self.r - score) / self.v - self.r

    def update_r(self, scores):
        self.r = float(np.percentile(scores, 100 * self.v))


def load_model_setting(task):
    """-> (Model, input_size, class_num, normed_mean, normed_std, is_discrete)  (utils_meta.py:5-35)"""
    if task == "mnist":
        return TASK_MODELS[task], (1, 28, 28), 10, np.array((0.1307,)), np.array((0.3081,)), False
    if task == "cifar10":
        return (TASK_MODELS[task], (3, 32, 32), 10, np.reshape(np.array((0.4914, 0.4822, 0.4465)), (3, 1, 1)),
                np.reshape(np.array((0.247, 0.243, 0.261)), (3, 1, 1)), False)
    if task == "audio":
        return TASK_MODELS[task], (16000,), 10, None, None, False
    if task == "rtNLP":
        return TASK_MODELS[task], (1, 10, 300), 1, None, None, True
    raise NotImplementedError(f"Unknown task {task}")


class CheckpointBank:
    """All (path, label) checkpoints resident on ``device``: path -> {name: tensor}."""

    def __init__(self, datasets: Sequence[Sequence[Tuple[str, int]]], device="cpu"):
        self.device = torch.device(device)
        self.params: Dict[str, Dict[str, torch.Tensor]] = {}
        self.missing: List[str] = []
        for ds in datasets:
            for path, _ in ds:
                if path in self.params or path in self.missing:
                    continue
                if not os.path.exists(path):
                    self.missing.append(path)
                    continue
                sd = torch.load(path, map_location="cpu", weights_only=True)
                self.params[path] = {k: v.to(self.device) for k, v in sd.items()}

    def filter(self, dataset):
        return [(p, y) for p, y in dataset if p in self.params]

    def __len__(self):
        return len(self.params)

    def stacked(self, paths: Sequence[str]) -> Dict[str, torch.Tensor]:
        """{name: [len(paths), *shape]} of the models in ``paths`` (cached per path tuple): the
        whole evaluation set as one batch of parameter tensors for a vmapped forward."""
        key = tuple(paths)
        cache = self.__dict__.setdefault("_stacked", {})
        if key not in cache:
            names = list(self.params[paths[0]].keys())
            cache[key] = {n: torch.stack([self.params[p][n] for p in paths]) for n in names}
        return cache[key]


class _EmbForward(nn.Module):
    """Routes forward() to the wrapped model's emb_forward() so functional_call can drive it."""

    def __init__(self, m):
        super().__init__()
        self.m = m

    def forward(self, x):
        return self.m.emb_forward(x)


def _call_method(module, params, fn, inp):
    """Run ``module.<fn>(inp)`` with the bank's resident tensors in place of its parameters."""
    if fn == "forward":
        return functional_call(module, params, (inp,), strict=False)
    return functional_call(_EmbForward(module), {"m." + k: v for k, v in params.items()}, (inp,), strict=False)


def _threshold(preds, threshold):
    return float(np.median(preds)) if threshold == "half" else threshold


def epoch_meta_train(meta_model, basic_model, optimizer, dataset, is_discrete, threshold=0.0, bank=None):
    from sklearn.metrics import roc_auc_score
    meta_model.train()
    basic_model.train()
    cum_loss, preds, labs = 0.0, [], []
    for i in np.random.permutation(len(dataset)):
        x, y = dataset[i]
        if bank is not None:
            out = _call_method(basic_model, bank.params[x], "emb_forward" if is_discrete else "forward",
                               meta_model.inp)
        else:
            basic_model.load_state_dict(torch.load(x, weights_only=True))
            out = basic_model.emb_forward(meta_model.inp) if is_discrete else basic_model.forward(meta_model.inp)
        score = meta_model.forward(out)
        l = meta_model.loss(score, y)
        optimizer.zero_grad()
        l.backward()
        optimizer.step()
        cum_loss += l.item()
        preds.append(score.item())
        labs.append(y)
    preds, labs = np.array(preds), np.array(labs)
    auc = roc_auc_score(labs, preds)
    acc = ((preds > _threshold(preds, threshold)) == labs).mean()
    return cum_loss / len(dataset), auc, acc


# MI355X_DP_MNTD_BATCHED=0 falls back to the reference's one-model-at-a-time evaluation
BATCHED_EVAL = os.environ.get("MI355X_DP_MNTD_BATCHED", "1") != "0"


@torch.no_grad()
def _eval_scores_batched(meta_model, basic_model, dataset, is_discrete, bank):
    """Every model of ``dataset`` in ONE vmapped forward over the bank's stacked parameters, then
    the meta-classifier over all of them at once -- no per-model launches or host syncs (the
    reference: one torch.load + forward + .item() per model, utils_meta.py:74-104).  Shadow models
    stay in train mode like the reference; dropout (CIFAR CNN) draws per model."""
    paths = [x for x, _ in dataset]
    labs = np.array([y for _, y in dataset])
    stacked = bank.stacked(paths)
    fn = "emb_forward" if is_discrete else "forward"
    outs = vmap(lambda p: _call_method(basic_model, p, fn, meta_model.inp), randomness="different")(stacked)
    if isinstance(meta_model, MetaClassifier):
        emb = F.relu(meta_model.fc(outs.reshape(len(paths), meta_model.N_in * meta_model.class_num)))
        scores = meta_model.output(emb).reshape(-1)
        target = torch.as_tensor(labs, dtype=scores.dtype, device=scores.device)
        losses = F.binary_cross_entropy_with_logits(scores, target, reduction="none").tolist()
    else:
        emb = F.relu(meta_model.fc(outs.reshape(len(paths), meta_model.N_in * meta_model.class_num)))
        scores = emb @ meta_model.w
        losses = []
    return scores.detach().cpu().numpy().astype(np.float64), labs, losses


@torch.no_grad()
def _eval_scores(meta_model, basic_model, dataset, is_discrete, bank):
    if bank is not None and BATCHED_EVAL and len(dataset) > 0:
        return _eval_scores_batched(meta_model, basic_model, dataset, is_discrete, bank)
    preds, labs, losses = [], [], []
    for x, y in dataset:
        if bank is not None:
            out = _call_method(basic_model, bank.params[x], "emb_forward" if is_discrete else "forward",
                               meta_model.inp)
        else:
            basic_model.load_state_dict(torch.load(x, weights_only=True))
            out = basic_model.emb_forward(meta_model.inp) if is_discrete else basic_model.forward(meta_model.inp)
        score = meta_model.forward(out)
        preds.append(score.item())
        labs.append(y)
        if isinstance(meta_model, MetaClassifier):
            losses.append(meta_model.loss(score, y).item())
    return np.array(preds), np.array(labs), losses


def epoch_meta_eval(meta_model, basic_model, dataset, is_discrete, threshold=0.0, bank=None):
    from sklearn.metrics import roc_auc_score
    meta_model.eval()
    basic_model.train()  # as the reference (utils_meta.py:76): shadow models in train mode
    preds, labs, losses = _eval_scores(meta_model, basic_model, dataset, is_discrete, bank)
    auc = roc_auc_score(labs, preds)
    acc = ((preds > _threshold(preds, threshold)) == labs).mean()
    return float(np.mean(losses)), auc, acc


def epoch_meta_train_oc(meta_model, basic_model, optimizer, dataset, is_discrete, bank=None):
    scores, cum_loss = [], 0.0
    for i in np.random.permutation(len(dataset)):
        x, y = dataset[i]
        assert y == 1
        if bank is not None:
            out = _call_method(basic_model, bank.params[x], "emb_forward" if is_discrete else "forward",
                               meta_model.inp)
        else:
            basic_model.load_state_dict(torch.load(x, weights_only=True))
            out = basic_model.emb_forward(meta_model.inp) if is_discrete else basic_model.forward(meta_model.inp)
        score = meta_model.forward(out)
        scores.append(score.item())
        loss = meta_model.loss(score)
        optimizer.zero_grad()
        loss.backward()
        optimizer.step()
        cum_loss += loss.item()
        meta_model.update_r(scores)
    return cum_loss / len(dataset)


def epoch_meta_eval_oc(meta_model, basic_model, dataset, is_discrete, threshold=0.0, bank=None):
    from sklearn.metrics import roc_auc_score
    preds, labs, _ = _eval_scores(meta_model, basic_model, dataset, is_discrete, bank)
    auc = roc_auc_score(labs, preds)
    acc = ((preds > _threshold(preds, threshold)) == labs).mean()
    return auc, acc
