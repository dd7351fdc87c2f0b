"""Loader for the in-tree native smddp backend extension."""
from __future__ import annotations

import importlib.util
import os

from ._smddp_build import EXT_NAME, ext_path

NATIVE_DIR = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "_native"))
_mod = None


def load():
    """Return the extension module, or None if it was not built."""
    global _mod
    if _mod is not None:
        return _mod
    path = ext_path(NATIVE_DIR)
    if not os.path.exists(path):
        return None
    import torch  # noqa: F401  (libtorch must be loaded first)
    spec = importlib.util.spec_from_file_location(EXT_NAME, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    _mod = mod
    return mod
