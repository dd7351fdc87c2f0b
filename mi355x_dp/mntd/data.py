"""MNTD datasets and settings (reference notebooks/code/utils_basic.py:7-91,
model_lib/{audio,rtNLP}_dataset.py).

``load_dataset_setting(task)`` returns the reference's 9-tuple.  Datasets come from the
torchvision compat layer (synthetic stand-ins written when the real files are absent:
no network).  rtNLP: the reference ships only raw ``rt-polarity.{pos,neg}`` and
expects preprocessed ``train_data.npy``/``dev_data.npy``/``dict.json``/
``saved_emb.npy``; ``build_rtnlp`` creates them from the raw text (tokenise, 10-token
windows, vocabulary, random 300-d embedding -- word2vec/gensim is unavailable, so the
embedding is random and documented as such).
"""
from __future__ import annotations

import json
import os
import re

import numpy as np
import torch
import torch.utils.data

from .models import TASK_MODELS
from .trojan import TROJ

USED_CLS = ["yes", "no", "up", "down", "left", "right", "on", "off", "stop", "go"]


def _tv():
    import importlib
    try:
        return importlib.import_module("torchvision")
    except ImportError:
        import sys
        sys.path.append(os.path.join(os.path.dirname(__file__), "..", "..", "compat"))
        return importlib.import_module("torchvision")


class SpeechCommand(torch.utils.data.Dataset):
    """Preprocessed Speech Commands (npy) restricted to the 10 used classes."""

    def __init__(self, split, path="./raw_data/speech_command/processed", all_classes=None):
        name = {0: "train", 1: "val", 2: "test"}[split]
        xs = np.load(os.path.join(path, f"{name}_data.npy"), allow_pickle=False)
        ys = np.load(os.path.join(path, f"{name}_label.npy"), allow_pickle=False)
        all_classes = all_classes or USED_CLS
        cls_map = {all_classes.index(c): i for i, c in enumerate(USED_CLS) if c in all_classes}
        keep = [i for i, y in enumerate(ys) if int(y) in cls_map]
        self.Xs = xs[keep]
        self.ys = [cls_map[int(ys[i])] for i in keep]

    def __len__(self):
        return len(self.ys)

    def __getitem__(self, idx):
        return torch.as_tensor(self.Xs[idx], dtype=torch.float32), self.ys[idx]


class RTNLP(torch.utils.data.Dataset):
    def __init__(self, train, path="./raw_data/rt_polarity/"):
        pre = "train" if train else "dev"
        self.Xs = np.load(os.path.join(path, f"{pre}_data.npy"), allow_pickle=False)
        self.ys = np.load(os.path.join(path, f"{pre}_label.npy"), allow_pickle=False)
        with open(os.path.join(path, "dict.json")) as f:
            info = json.load(f)
        self.tok2idx, self.idx2tok = info["tok2idx"], info["idx2tok"]

    def __len__(self):
        return len(self.ys)

    def __getitem__(self, idx):
        return torch.as_tensor(self.Xs[idx], dtype=torch.long), int(self.ys[idx])


def build_rtnlp(raw_dir="./raw_data/rt_polarity", max_len=10, dim=300, dev_frac=0.1, seed=0):
    """Preprocess raw rt-polarity text into the files RTNLP/RTNLPCNN expect."""
    rng = np.random.default_rng(seed)
    docs = []
    for fname, lab in (("rt-polarity.pos", 1), ("rt-polarity.neg", 0)):
        with open(os.path.join(raw_dir, fname), "rb") as f:
            for line in f.read().decode("latin-1").splitlines():
                toks = re.findall(r"[a-z0-9']+", line.lower())
                if toks:
                    docs.append((toks, lab))
    vocab = {"<pad>": 0, "<unk>": 1}
    for toks, _ in docs:
        for t in toks:
            vocab.setdefault(t, len(vocab))
    X = np.zeros((len(docs), max_len), dtype=np.int64)
    y = np.zeros(len(docs), dtype=np.int64)
    for i, (toks, lab) in enumerate(docs):
        ids = [vocab[t] for t in toks[:max_len]]
        X[i, :len(ids)] = ids
        y[i] = lab
    perm = rng.permutation(len(docs))
    n_dev = int(len(docs) * dev_frac)
    dev, tr = perm[:n_dev], perm[n_dev:]
    np.save(os.path.join(raw_dir, "train_data.npy"), X[tr])
    np.save(os.path.join(raw_dir, "train_label.npy"), y[tr])
    np.save(os.path.join(raw_dir, "dev_data.npy"), X[dev])
    np.save(os.path.join(raw_dir, "dev_label.npy"), y[dev])
    emb = rng.normal(0, 0.1, (max(len(vocab), 18000), dim)).astype(np.float32)
    emb[0] = 0
    np.save(os.path.join(raw_dir, "saved_emb.npy"), emb)
    with open(os.path.join(raw_dir, "dict.json"), "w") as f:
        json.dump({"tok2idx": vocab, "idx2tok": {v: k for k, v in vocab.items()}}, f)
    return len(docs), len(vocab)


def load_dataset_setting(task, root="./raw_data/"):
    """-> (BATCH_SIZE, N_EPOCH, trainset, testset, is_binary, need_pad, Model, troj_gen_func, random_troj_setting)"""
    if task in ("mnist", "cifar10"):
        tv = _tv()
        tf = tv.transforms.Compose([tv.transforms.ToTensor()])
        cls = tv.datasets.MNIST if task == "mnist" else tv.datasets.CIFAR10
        trainset = cls(root=root, train=True, download=True, transform=tf)
        testset = cls(root=root, train=False, download=False, transform=tf)
        bs, ne, is_binary, need_pad = 100, 100, False, False
    elif task == "audio":
        trainset, testset = SpeechCommand(0), SpeechCommand(2)
        bs, ne, is_binary, need_pad = 100, 100, False, False
    elif task == "rtNLP":
        trainset, testset = RTNLP(True), RTNLP(False)
        bs, ne, is_binary, need_pad = 64, 50, True, True
    else:
        raise NotImplementedError(f"Unknown task {task}")
    setting, stamp = TROJ[task]
    return bs, ne, trainset, testset, is_binary, need_pad, TASK_MODELS[task], stamp, setting


class BackdoorDataset(torch.utils.data.Dataset):
    """Clean samples ``choice`` followed by ``inject_p * |choice|`` poisoned ones (``mal_only``:
    poisoned only, for attack-success evaluation).  utils_basic.py:54-91."""

    def __init__(self, src_dataset, atk_setting, troj_gen_func, choice=None, mal_only=False, need_pad=False):
        self.src_dataset = src_dataset
        self.atk_setting = atk_setting
        self.troj_gen_func = troj_gen_func
        self.need_pad = need_pad
        self.mal_only = mal_only
        self.choice = np.arange(len(src_dataset)) if choice is None else choice
        self.mal_choice = np.random.choice(self.choice, int(len(self.choice) * atk_setting[5]), replace=False)

    def __len__(self):
        return len(self.mal_choice) if self.mal_only else len(self.choice) + len(self.mal_choice)

    def __getitem__(self, idx):
        if not self.mal_only and idx < len(self.choice):
            X, y = self.src_dataset[self.choice[idx]]
            if self.need_pad:
                X = torch.cat([X, torch.zeros(self.atk_setting[0], dtype=torch.long)], dim=0)
            return X, y
        j = self.mal_choice[idx] if self.mal_only else self.mal_choice[idx - len(self.choice)]
        X, y = self.src_dataset[j]
        return self.troj_gen_func(X, y, self.atk_setting)
