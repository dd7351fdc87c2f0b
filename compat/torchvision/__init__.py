"""Minimal torchvision compatibility package for mi355x_dp (torchvision itself is not
installed in this environment).  Provides exactly what the workshop code imports:
``datasets.CIFAR10/MNIST``, ``transforms.{Compose,ToTensor,Normalize,RandomCrop,
RandomHorizontalFlip,...}``, ``models.resnet18/34/50/101/152, vit_b_16`` (backed by
mi355x_dp's native-kernel models, identical parameter names) and ``utils.make_grid``.

It is only put on ``sys.path`` by the mi355x_dp launcher / local-mode estimator and
never shadows a real torchvision install (see mi355x_dp.compat_path)."""
__version__ = "0.0.0+mi355x_dp.compat"

from . import datasets, models, transforms, utils  # noqa: F401,E402
