"""Utilities: logging (reference line formats), checkpoint/resume, environment helpers."""
from .checkpoint import load_checkpoint, save_checkpoint, save_model  # noqa: F401
from .logging import get_logger  # noqa: F401
