"""Loader for the in-tree native bucket reducer (csrc/ddp/reducer.cpp)."""
from __future__ import annotations

import importlib.util
import os

from ._smddp_build import ext_path

NATIVE_DIR = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "_native"))
EXT_NAME = "_reducer_ext"
_mod = None


def load():
    """Return the extension module, or None if it was not built."""
    global _mod
    if _mod is not None:
        return _mod
    if os.environ.get("MI355X_DP_PY_REDUCER") == "1":
        return None
    path = ext_path(NATIVE_DIR, EXT_NAME)
    if not os.path.exists(path):
        return None
    import torch  # noqa: F401  (libtorch / c10d must be loaded first)
    import torch.distributed  # noqa: F401
    spec = importlib.util.spec_from_file_location(EXT_NAME, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    _mod = mod
    return mod
