"""The ``smddp`` process-group backend (SMDDP-equivalent, reference gpu.py:16-23,
SURVEY.md §2.2 C25 / §5.8).

``import smdistributed.dataparallel.torch.torch_smddp`` (our compat shim) calls
``register()``, after which the reference's ``dist.init_process_group(backend='smddp')``
works unmodified.  The creator:

  1. binds the rank to its GPU *before* anything else (``LOCAL_RANK``): the
     reference moves the model to "cuda" and wraps DDP before calling
     ``set_device`` (gpu.py:145-153), which only works because SMDDP binds the
     device at init;
  2. returns the native C++ backend (``csrc/comm/smddp_backend.cpp``: RCCL
     communicator on its own high-priority HIP stream, event-ordered with the
     caller's stream, plus xGMI-aware bucket chunking).  A missing build is an
     error, not a silent fallback; ``MI355X_DP_SMDDP_IMPL=nccl`` deliberately
     selects torch's RCCL ``ProcessGroupNCCL`` instead;
  3. on a host with no GPU (CPU tests, gloo plumbing) returns a gloo backend
     bound to the loopback interface so the same user code runs.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

BACKEND_NAME = "smddp"
_registered = False


def _gpu_count() -> int:
    try:
        return torch.cuda.device_count()
    except Exception:
        return 0


def bind_local_device():
    n = _gpu_count()
    if n <= 0:
        return None
    local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("OMPI_COMM_WORLD_LOCAL_RANK", "0")))
    dev = local_rank % n
    if os.environ.get("MI355X_DP_SMDDP_DEVICE"):  # testing: several ranks sharing one GPU (IPC path)
        dev = int(os.environ["MI355X_DP_SMDDP_DEVICE"])
    torch.cuda.set_device(dev)
    return dev


def _gloo(store, rank, world_size, timeout):
    opts = dist.ProcessGroupGloo._Options()
    opts._timeout = timeout
    host = os.environ.get("MI355X_DP_GLOO_HOST", "127.0.0.1")
    opts._devices = [dist.ProcessGroupGloo.create_device(hostname=host)]
    return dist.ProcessGroupGloo(store, rank, world_size, opts)


def create_backend(store, rank, world_size, timeout):
    dev = bind_local_device()
    if dev is None:
        return _gloo(store, rank, world_size, timeout)
    if os.environ.get("MI355X_DP_SMDDP_IMPL", "native") == "native":
        # the native backend is the product: a missing / broken build fails loudly instead of
        # silently running torch's ProcessGroupNCCL (MI355X_DP_SMDDP_IMPL=nccl selects that on purpose)
        from . import _smddp_native
        mod = _smddp_native.load()
        if mod is None:
            raise RuntimeError("smddp: native backend extension (_smddp_native_ext) is not built; run "
                               "`python -m mi355x_dp.build` or set MI355X_DP_SMDDP_IMPL=nccl")
        if (os.environ.get("MI355X_DP_SMDDP_IPC") == "1" or os.environ.get("MI355X_DP_SMDDP_IPC_ONLY") == "1"
                or int(os.environ.get("MI355X_DP_COMM_EMULATE", "0") or 0) > 1):
            # the one-shot IPC all-reduce kernel and the world-1 ring emulation live in the HIP
            # kernel library
            from mi355x_dp.ops import _lib
            _lib.load(True)
            os.environ.setdefault("MI355X_DP_KERNELS_LIB", _lib.KERNEL_LIB)
        secs = timeout.total_seconds() if isinstance(timeout, datetime.timedelta) else float(timeout)
        return mod.create_backend(store, rank, world_size, dev, secs)
    return dist.ProcessGroupNCCL(store, rank, world_size, timeout)


def register():
    """Idempotently register the ``smddp`` backend name with torch.distributed."""
    global _registered
    if _registered or BACKEND_NAME in dist.Backend.backend_list:
        _registered = True
        return
    dist.Backend.register_backend(BACKEND_NAME, create_backend, extended_api=False, devices=["cpu", "cuda"])
    _registered = True
