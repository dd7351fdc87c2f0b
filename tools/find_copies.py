"""Debug: which Python call sites issue device copies in a ResNet-50 training step?  Wraps
Tensor.copy_/clone/contiguous/to and counts CUDA-tensor calls by call site over 2 steps."""
import collections
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mi355x_dp.models import resnet50  # noqa: E402
from mi355x_dp.ops import augment, cross_entropy  # noqa: E402
from mi355x_dp.parallel import DataParallel, FlatSGD  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
eng = DataParallel(resnet50().to(dev))
opt = FlatSGD(eng, lr=0.01, momentum=0.9, weight_decay=1e-4)
images = torch.randint(0, 256, (256, 224, 224, 3), dtype=torch.uint8, device=dev)
labels = torch.randint(0, 1000, (256,), device=dev)
x = torch.empty((256, 8, 224, 224), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)


def step(i):
    augment(images, 8, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), pad=0, flip=True, seed=i, out=x)
    eng.zero_grad()
    loss = cross_entropy(eng(x), labels)
    loss.backward()
    opt.step()


step(0)
torch.cuda.synchronize()
counts = collections.Counter()
orig = {}
for name in ("copy_", "clone", "contiguous", "to", "zero_", "fill_"):
    orig[name] = getattr(torch.Tensor, name)

    def make(name):
        f = orig[name]

        def w(self, *a, **k):
            if self.is_cuda:
                st = traceback.extract_stack(limit=6)[:-1]
                site = " <- ".join(f"{os.path.basename(fr.filename)}:{fr.lineno}" for fr in reversed(st[-3:]))
                counts[(name, site)] += 1
            return f(self, *a, **k)
        return w
    setattr(torch.Tensor, name, make(name))
for i in range(2):
    step(1 + i)
torch.cuda.synchronize()
for (name, site), n in counts.most_common(40):
    print(f"{n / 2:6.1f}/step  {name:10s} {site}")
