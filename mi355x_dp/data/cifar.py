"""CIFAR-10 on-disk format: reader (safe) and synthetic writer.

Layout is the official ``cifar-10-batches-py`` directory (data_batch_1..5,
test_batch, batches.meta: pickled dicts with ``b'data'`` uint8 [N, 3072] in
CHW order and ``b'labels'``), which is what the reference scripts read through
``torchvision.datasets.CIFAR10(root=SM_CHANNEL_TRAIN)`` (reference
cifar10-distributed-smddp-gpu.py:70-73).

There is no network here, so ``write_synthetic_cifar10`` produces a
*learnable* stand-in of the same shape: each class is a fixed random
low-frequency colour template mixed with a distractor of another class, heavy
noise and random shifts, with a quarter of the samples ambiguous -- so accuracy
curves rise over epochs and saturate below 1.0 (see ``_make_split``).

Reading uses a restricted unpickler (plain containers + numpy array
reconstruction only): pickles are never loaded with an unrestricted loader.
"""
from __future__ import annotations

import io
import os
import pickle

import numpy as np

BASE = "cifar-10-batches-py"
TRAIN_FILES = [f"data_batch_{i}" for i in range(1, 6)]
TEST_FILE = "test_batch"
META_FILE = "batches.meta"
CLASSES = ["airplane", "automobile", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck"]

_ALLOWED = {
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"), ("builtins", "bytes"), ("_codecs", "encode"),
}


class SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name}")


def safe_load_pickle(path):
    with open(path, "rb") as f:
        return SafeUnpickler(f, encoding="bytes").load()


def load_batch(path):
    d = safe_load_pickle(path)
    data = d.get(b"data", d.get("data"))
    labels = d.get(b"labels", d.get("labels", d.get(b"fine_labels")))
    return np.asarray(data, dtype=np.uint8).reshape(-1, 3, 32, 32), np.asarray(labels, dtype=np.int64)


def load_cifar10(root, train=True):
    """-> (images uint8 [N,32,32,3] HWC, labels int64 [N])."""
    base = os.path.join(root, BASE)
    files = TRAIN_FILES if train else [TEST_FILE]
    xs, ys = [], []
    for f in files:
        x, y = load_batch(os.path.join(base, f))
        xs.append(x)
        ys.append(y)
    x = np.concatenate(xs).transpose(0, 2, 3, 1).copy()
    return x, np.concatenate(ys)


def exists(root):
    base = os.path.join(root, BASE)
    return all(os.path.exists(os.path.join(base, f)) for f in TRAIN_FILES + [TEST_FILE])


def _class_templates(rng):
    t = np.zeros((10, 32, 32, 3), np.float32)
    yy, xx = np.mgrid[0:32, 0:32] / 32.0
    for c in range(10):
        for ch in range(3):
            fx, fy, ph = rng.uniform(0.5, 3.0), rng.uniform(0.5, 3.0), rng.uniform(0, 2 * np.pi)
            t[c, :, :, ch] = 0.5 + 0.35 * np.sin(2 * np.pi * (fx * xx + fy * yy) + ph)
    return t


def _make_split(rng, templates, n, ambiguous=0.25):
    """Images of class c: 0.6 x (template c + a weaker distractor template of another class) +
    heavy noise, rolled by up to +-8 pixels.  A fraction ``ambiguous`` of the samples is drawn
    from a random OTHER class's template but keeps label c, so the Bayes accuracy is about
    1 - 0.9 * ambiguous (~0.78) and the curve saturates like real CIFAR-10 (the reference
    reaches 0.71 after 15 epochs, nb2:2559) instead of hitting 1.00 in the first epoch."""
    labels = rng.integers(0, 10, n)
    src = np.where(rng.random(n) < ambiguous, rng.integers(0, 10, n), labels)
    other = (src + rng.integers(1, 10, n)) % 10
    w = rng.uniform(0.3, 0.7, (n, 1, 1, 1)).astype(np.float32)
    imgs = 0.5 + 0.6 * ((templates[src] - 0.5) + w * (templates[other] - 0.5))
    imgs += rng.normal(0, 0.35, (n, 32, 32, 3)).astype(np.float32)
    shifts = rng.integers(-8, 9, (n, 2))
    for i in range(n):  # random translations keep the task non-trivial
        imgs[i] = np.roll(imgs[i], tuple(shifts[i]), axis=(0, 1))
    return (np.clip(imgs, 0, 1) * 255).astype(np.uint8), labels


def write_synthetic_cifar10(root, n_train=None, n_test=None, seed=0):
    """Write a synthetic dataset in the official layout; returns the batches dir.  Sizes default
    to the real 50000 / 10000 (MI355X_DP_SYNTH_CIFAR_TRAIN / _TEST override them, e.g. to keep
    a verbatim notebook run short on CPU)."""
    if n_train is None:
        n_train = int(os.environ.get("MI355X_DP_SYNTH_CIFAR_TRAIN", "50000"))
    if n_test is None:
        n_test = int(os.environ.get("MI355X_DP_SYNTH_CIFAR_TEST", "10000"))
    base = os.path.join(root, BASE)
    os.makedirs(base, exist_ok=True)
    rng = np.random.default_rng(seed)
    templates = _class_templates(rng)
    per = [n_train // 5 + (1 if i < n_train % 5 else 0) for i in range(5)]
    for fname, n in list(zip(TRAIN_FILES, per)) + [(TEST_FILE, n_test)]:
        x, y = _make_split(rng, templates, n)
        d = {b"batch_label": fname.encode(), b"labels": [int(v) for v in y],
             b"data": x.transpose(0, 3, 1, 2).reshape(n, 3072).copy(),
             b"filenames": [f"synthetic_{i}.png".encode() for i in range(n)]}
        with open(os.path.join(base, fname), "wb") as f:
            pickle.dump(d, f, protocol=2)
    with open(os.path.join(base, META_FILE), "wb") as f:
        pickle.dump({b"label_names": [c.encode() for c in CLASSES], b"num_cases_per_batch": per[0],
                     b"num_vis": 3072}, f, protocol=2)
    with open(os.path.join(base, "SYNTHETIC"), "w") as f:
        f.write("synthetic stand-in for CIFAR-10 (no network access); class templates + distractors + noise, "
                "25% ambiguous samples\n")
    return base
