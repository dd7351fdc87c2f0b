"""torchvision.datasets subset: CIFAR10 and MNIST.

* CIFAR10 reads the official ``cifar-10-batches-py`` layout through a restricted
  unpickler (mi355x_dp.data.cifar).  ``download=True`` cannot reach the network
  here: it writes a *synthetic* learnable stand-in of the exact on-disk layout
  instead and logs that it did so.
* MNIST reads raw IDX files (``MNIST/raw/*-ubyte``); ``download=True`` likewise
  writes a synthetic IDX set of the official shape.
"""
import gzip
import logging
import os

import numpy as np
import torch

from mi355x_dp.data import cifar as _cifar

try:
    from PIL import Image
except Exception:  # pragma: no cover
    Image = None

log = logging.getLogger("torchvision.compat")


class VisionDataset(torch.utils.data.Dataset):
    def __init__(self, root, transform=None, target_transform=None):
        self.root = os.path.expanduser(root) if isinstance(root, str) else root
        self.transform = transform
        self.target_transform = target_transform


class CIFAR10(VisionDataset):
    base_folder = _cifar.BASE
    classes = _cifar.CLASSES

    def __init__(self, root, train=True, transform=None, target_transform=None, download=False):
        super().__init__(root, transform, target_transform)
        self.train = train
        if not _cifar.exists(self.root):
            if not download:
                raise RuntimeError("Dataset not found or corrupted. You can use download=True to download it")
            log.warning("no network: writing a synthetic CIFAR-10 stand-in under %s", self.root)
            _cifar.write_synthetic_cifar10(self.root)
        self.data, targets = _cifar.load_cifar10(self.root, train=train)
        self.targets = [int(t) for t in targets]
        self.class_to_idx = {c: i for i, c in enumerate(self.classes)}

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        img, target = self.data[index], self.targets[index]
        img = Image.fromarray(img) if Image is not None else img
        if self.transform is not None:
            img = self.transform(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, target

    def __getitems__(self, indices):
        """Batched fetch used by DataLoader auto-collation: the whole batch is transformed
        with a few vectorised ops (transforms.batch_apply) instead of one PIL round trip per
        image; falls back to per-image __getitem__ for pipelines it does not recognise."""
        return _batched_items(self, self.data, indices)


def _batched_items(ds, data, indices):
    from torchvision import transforms as _T
    idx = np.asarray(indices, dtype=np.int64)
    batch = None
    if ds.transform is not None and ds.target_transform is None and len(idx):
        cache = ds.__dict__.setdefault("_batch_cache", {})
        batch = _T.batch_apply(ds.transform, (data, idx), cache=cache)
    if batch is None:
        return [ds[int(i)] for i in idx]
    tg = ds.targets
    labels = [int(tg[int(i)]) for i in idx]
    return list(zip(batch.unbind(0), labels))


def _read_idx(path):
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        data = f.read()
    magic = int.from_bytes(data[0:4], "big")
    nd = magic & 0xFF
    dims = [int.from_bytes(data[4 + 4 * i:8 + 4 * i], "big") for i in range(nd)]
    return np.frombuffer(data, dtype=np.uint8, offset=4 + 4 * nd).reshape(dims)


def _write_idx(path, arr):
    arr = np.asarray(arr, dtype=np.uint8)
    with open(path, "wb") as f:
        f.write((0x0800 | arr.ndim).to_bytes(4, "big"))
        for d in arr.shape:
            f.write(int(d).to_bytes(4, "big"))
        f.write(arr.tobytes())


def write_synthetic_mnist(raw_dir, n_train=60000, n_test=10000, seed=0):
    os.makedirs(raw_dir, exist_ok=True)
    rng = np.random.default_rng(seed)
    templates = (rng.random((10, 28, 28)) > 0.75).astype(np.float32)
    for prefix, n in (("train", n_train), ("t10k", n_test)):
        y = rng.integers(0, 10, n)
        x = templates[y] * 200 + rng.normal(0, 25, (n, 28, 28))
        _write_idx(os.path.join(raw_dir, f"{prefix}-images-idx3-ubyte"), np.clip(x, 0, 255))
        _write_idx(os.path.join(raw_dir, f"{prefix}-labels-idx1-ubyte"), y)
    with open(os.path.join(raw_dir, "SYNTHETIC"), "w") as f:
        f.write("synthetic stand-in for MNIST (no network access)\n")


class MNIST(VisionDataset):
    classes = [f"{i} - {w}" for i, w in enumerate(["zero", "one", "two", "three", "four", "five", "six", "seven",
                                                   "eight", "nine"])]

    def __init__(self, root, train=True, transform=None, target_transform=None, download=False):
        super().__init__(root, transform, target_transform)
        self.train = train
        raw = os.path.join(self.root, "MNIST", "raw")
        prefix = "train" if train else "t10k"
        img_p = os.path.join(raw, f"{prefix}-images-idx3-ubyte")
        if not (os.path.exists(img_p) or os.path.exists(img_p + ".gz")):
            if not download:
                raise RuntimeError("Dataset not found. You can use download=True to download it")
            log.warning("no network: writing a synthetic MNIST stand-in under %s", raw)
            write_synthetic_mnist(raw)
        pick = lambda p: p if os.path.exists(p) else p + ".gz"  # noqa: E731
        self.data = torch.from_numpy(_read_idx(pick(img_p)).copy())
        self.targets = torch.from_numpy(
            _read_idx(pick(os.path.join(raw, f"{prefix}-labels-idx1-ubyte"))).astype(np.int64))

    def __len__(self):
        return len(self.data)

    def __getitem__(self, index):
        img, target = self.data[index], int(self.targets[index])
        img = Image.fromarray(img.numpy(), mode="L") if Image is not None else img
        if self.transform is not None:
            img = self.transform(img)
        if self.target_transform is not None:
            target = self.target_transform(target)
        return img, target

    def __getitems__(self, indices):
        return _batched_items(self, self.data, indices)
