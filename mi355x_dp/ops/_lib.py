"""Loader for the in-tree native kernel library (``libmi355x_kernels.so``).

The HIP/CDNA4 kernels under ``csrc/kernels/*.hip`` are compiled for gfx950 into
one shared object with a plain C ABI (see ``csrc/kernels/api.h``).  Python binds
it with ctypes: every launcher takes raw device pointers plus the HIP stream
handle of ``torch.cuda.current_stream()``, so kernels are stream-ordered with
PyTorch's own work and are captured by ``torch.cuda.CUDAGraph`` like any other
launch.

Policy: when a tensor lives on the GPU the native library is REQUIRED.  There is
no silent fallback to an eager PyTorch implementation on the device; the CPU
reference implementations in ``mi355x_dp.ops`` exist only for host tensors
(tests, the gloo CPU configuration).
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE_DIR = os.path.normpath(os.path.join(_HERE, "..", "_native"))
KERNEL_LIB = os.path.join(NATIVE_DIR, "libmi355x_kernels.so")
# MI355X_DP_DEBUG_KERNELS=1: the -DMI_DEBUG build (device bounds asserts; `python -m mi355x_dp.build
# kernels --debug`).  MI355X_DP_SYNC_CHECK=1: synchronise after every native call so an
# asynchronous device fault is reported against the kernel that caused it.
if os.environ.get("MI355X_DP_DEBUG_KERNELS") == "1":
    KERNEL_LIB = os.path.join(NATIVE_DIR, "libmi355x_kernels_debug.so")
elif os.environ.get("MI355X_DP_KERNEL_VARIANT"):  # A/B builds: mi355x_dp.build.build_kernels(variant=...)
    KERNEL_LIB = os.path.join(NATIVE_DIR, f"libmi355x_kernels_{os.environ['MI355X_DP_KERNEL_VARIANT']}.so")
SYNC_CHECK = os.environ.get("MI355X_DP_SYNC_CHECK") == "1"

_lock = threading.Lock()
_lib = None
_load_error = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_float = ctypes.c_float

# name -> argtypes.  Every launcher returns int (hipError_t).
_SIGNATURES = {}


def signature(name, *argtypes, restype=None):
    _SIGNATURES[name] = (list(argtypes), restype if restype is not None else c_int)


def _bind(lib):
    for name, (argtypes, restype) in _SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            raise RuntimeError(f"native kernel library is stale: missing symbol {name}; rebuild with `python -m mi355x_dp.build`")
        fn.argtypes = argtypes
        fn.restype = restype


def load(required: bool = True):
    """Return the ctypes handle, or None (only when ``required`` is False)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(KERNEL_LIB):
            _load_error = f"{KERNEL_LIB} not built (run `python -m mi355x_dp.build`)"
        else:
            try:
                lib = ctypes.CDLL(KERNEL_LIB, mode=ctypes.RTLD_GLOBAL)
                _bind(lib)
                _lib = lib
                return _lib
            except OSError as e:  # pragma: no cover - depends on the box
                _load_error = f"failed to load {KERNEL_LIB}: {e}"
    if required:
        raise RuntimeError("mi355x_dp native kernels unavailable on a GPU tensor: " + str(_load_error))
    return None


def available() -> bool:
    return load(required=False) is not None


def check(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")


def stream_of(t=None):
    import torch
    dev = t.device if t is not None else None
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# BatchNorm entry points whose tall-slab finalize uses the per-stream arrival counters of
# mi_bn_init_counters(): the table is allocated on the first such call (the GPU is initialised by
# then, and GraphedStep's eager warm-up makes it happen before any capture).  A process that later
# uses another device simply takes the counter-free two-launch path there.
_BN_COUNTER_USERS = frozenset(("mi_bn_fwd_train", "mi_bn_bwd_train", "mi_bn_bwd_train_pre"))
_bn_counters_pending = [True]


def call(name, *args):
    lib = load(True)
    if _bn_counters_pending[0] and name in _BN_COUNTER_USERS:
        _bn_counters_pending[0] = False
        check(lib.mi_bn_init_counters(), "mi_bn_init_counters")
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")
    if SYNC_CHECK:
        import torch
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:
            raise RuntimeError(f"{name}: device error after launch ({e})") from e
