"""Engine-backed ``torch.nn.parallel.DistributedDataParallel`` for unmodified user scripts
(SURVEY.md §7.1 decision 2(b)).

The reference GPU script wraps its model in the stock class and drives it with stock
``optim.SGD`` (cifar10-distributed-smddp-gpu.py:145-168).  Stock DDP on top of our kernels
copies every gradient into its own bucket tensors and back, fills and rescales per parameter, and
stock SGD then changes the fp32 parameters behind the bf16 compute copies -- on one MI355X that was
~300 small ATen launches per step and a host-bound loop with the GPU busy 24 % of the time
(profiles/reference_unmodified_job.md).

``install()`` (run by the ``smdistributed.dataparallel.torch.torch_smddp`` import shim, i.e. only
when a script opts into SMDDP) replaces the ``torch.nn.parallel.DistributedDataParallel`` name with
this factory.  For a model built from the framework's native layers (compat ``torchvision``
ResNets / ViT) on a GPU it returns the flat-buffer engine (``DataParallel(foreign_optimizer=True)``):
gradients written straight into one flat fp32 buffer by the backward kernels, bucket collectives
launched by the C++ reducer during backward, the averaged result in ``p.grad`` when ``backward()``
returns, ``state_dict`` keys prefixed ``module.`` exactly like torch DDP (``model.pth`` unchanged).
Anything else -- a stock ``nn`` model such as the script's ``Net``, CPU modules, unsupported DDP
options -- gets the stock class.  ``MI355X_DP_ENGINE_DDP=0`` disables the substitution.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
import torch.nn as nn

_STOCK = None  # torch's own class, kept before install() replaces the public name
# torch DDP keyword arguments the engine honours (their semantics: DataParallel.__init__)
_ACCEPTED = {"device_ids", "output_device", "dim", "broadcast_buffers", "process_group", "bucket_cap_mb",
             "find_unused_parameters", "gradient_as_bucket_view", "static_graph"}


def stock_ddp():
    return _STOCK if _STOCK is not None else torch.nn.parallel.DistributedDataParallel


def eligible(module: nn.Module, kwargs) -> bool:
    """The engine path: enabled, every DDP option one the engine honours, all trainable
    parameters on one CUDA device, and at least one native conv / linear layer in the model."""
    mode = os.environ.get("MI355X_DP_ENGINE_DDP", "1")
    if mode == "0":
        return False
    if set(kwargs) - _ACCEPTED:
        return False
    params = [p for p in module.parameters() if p.requires_grad]
    # "force": CPU modules too (tests of the substitution on machines without a GPU)
    if not params or any((p.device.type != "cuda" and mode != "force") or p.device != params[0].device
                         for p in params):
        return False
    if any(p.dtype != torch.float32 for p in params):
        return False
    from mi355x_dp.models.layers import Conv2d, Linear
    return any(isinstance(m, (Conv2d, Linear)) for m in module.modules())


class _FactoryMeta(type):
    """Keeps the public name behaving like a class for user code:

    * ``isinstance(m, torch.nn.parallel.DistributedDataParallel)`` -- the usual way scripts and
      libraries decide to unwrap ``.module`` -- holds for both things the factory returns (the
      engine and the stock fallback), and ``issubclass`` likewise;
    * ``class MyDDP(torch.nn.parallel.DistributedDataParallel)`` written after the shim is
      imported derives from torch's own class, so the subclass keeps stock semantics."""

    def __new__(mcls, name, bases, ns, **kw):
        if any(isinstance(b, _FactoryMeta) for b in bases) and ns.get("_mi355x_factory") is None:
            stock = stock_ddp()
            bases = tuple(stock if isinstance(b, _FactoryMeta) else b for b in bases)
            return type(stock)(name, bases, ns, **kw)
        return super().__new__(mcls, name, bases, ns, **kw)

    def __instancecheck__(cls, obj):
        from .ddp import DataParallel
        return isinstance(obj, (stock_ddp(), DataParallel))

    def __subclasscheck__(cls, sub):
        from .ddp import DataParallel
        return sub is cls or issubclass(sub, (stock_ddp(), DataParallel))


class DistributedDataParallel(metaclass=_FactoryMeta):
    """Factory standing in for ``torch.nn.parallel.DistributedDataParallel`` (see module doc)."""

    _mi355x_factory = True

    def __new__(cls, module, *args, **kwargs):
        if args:  # positional device_ids etc.: torch's signature order
            names = ["device_ids", "output_device", "dim", "broadcast_buffers", "process_group", "bucket_cap_mb",
                     "find_unused_parameters", "check_reduction", "gradient_as_bucket_view", "static_graph"]
            kwargs = {**dict(zip(names, args)), **kwargs}
        if eligible(module, kwargs):
            from .ddp import DataParallel
            kw = dict(kwargs)
            kw.setdefault("broadcast_buffers", True)
            eng = DataParallel(module, foreign_optimizer=True, **kw)
            if eng.rank == 0:
                # precision honesty: the reference trains in fp32 (TF32-class
                # convs on A100); the engine's native kernels compute in bf16
                from mi355x_dp.ops.fp32 import COMPUTE_FP32
                cd = "fp32 (MFMA f32 operands, exact fp32)" if COMPUTE_FP32 else "bf16 (MFMA, fp32 accumulation)"
                print(f"[mi355x_dp] DistributedDataParallel -> native engine: compute dtype {cd}, "
                      "fp32 master weights, fp32 gradients and all-reduce "
                      f"({len(eng.buckets)} buckets, world {eng.world_size})", flush=True)
            return eng
        return stock_ddp()(module, **kwargs)


def install():
    """Idempotently point ``torch.nn.parallel.DistributedDataParallel`` at the factory."""
    global _STOCK
    import torch.nn.parallel as tnp
    if _STOCK is None:
        _STOCK = tnp.DistributedDataParallel
    tnp.DistributedDataParallel = DistributedDataParallel


def uninstall():
    import torch.nn.parallel as tnp
    if _STOCK is not None:
        tnp.DistributedDataParallel = _STOCK


def is_engine(model) -> bool:
    from .ddp import DataParallel
    return isinstance(model, DataParallel)


__all__ = ["DistributedDataParallel", "install", "uninstall", "eligible", "stock_ddp", "is_engine", "dist"]
