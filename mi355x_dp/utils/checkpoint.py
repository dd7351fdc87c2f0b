"""Checkpointing.

* ``save_model(model, model_dir)`` -- the reference's artifact: rank-0
  ``torch.save(model.state_dict(), <model_dir>/model.pth)`` (plain state_dict, NCHW
  contiguous tensors; a DDP/DataParallel wrapper keeps its ``module.`` prefix exactly as
  in cifar10-distributed-smddp-gpu.py:205-208).
* ``save_checkpoint`` / ``load_checkpoint`` -- resumable training state the reference
  lacks: model + optimizer (flat momentum buffer) + step/epoch + RNG states, written
  atomically by rank 0 to a separate file (never changes model.pth), restored on every
  rank (map_location to the local device) with ``weights_only=True``.  An optimizer whose state is
  sharded over ranks (``FlatSGD`` under ``DataParallel(shard_optimizer=True)``: each rank holds the
  momentum of its own shards only) is written by EVERY rank to ``<path>.optim-rank<r>-of-<w>``;
  the main file records the world size and loading checks it.
"""
from __future__ import annotations

import os
import tempfile
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist


def _rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def save_model(model: torch.nn.Module, model_dir: str, filename: str = "model.pth") -> Optional[str]:
    if _rank() != 0:
        return None
    os.makedirs(model_dir, exist_ok=True)
    path = os.path.join(model_dir, filename)
    sd = {k: (v.detach().cpu().contiguous() if isinstance(v, torch.Tensor) else v)
          for k, v in model.state_dict().items()}
    _atomic_save(sd, path)
    return path


def _atomic_save(obj, path):
    d = os.path.dirname(os.path.abspath(path))
    # no leading dot: torch's zip writer derives the archive name from the file name and rejects
    # an empty stem ("invalid file name")
    fd, tmp = tempfile.mkstemp(dir=d, prefix="tmp_ckpt_", suffix=".partial")
    os.close(fd)
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def optim_shard_path(path: str, rank: int, world: int) -> str:
    return f"{path}.optim-rank{rank}-of-{world}"


def save_checkpoint(path: str, model: torch.nn.Module, optimizer=None, step: int = 0, epoch: int = 0,
                    extra: Optional[Dict[str, Any]] = None) -> Optional[str]:
    osd = optimizer.state_dict() if optimizer is not None else None
    sharded = isinstance(osd, dict) and "shard" in osd
    if sharded:
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        _atomic_save(osd, optim_shard_path(path, _rank(), _world()))
    if _rank() != 0:
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
        return None
    state = {
        "model": {k: v.detach().cpu().contiguous() for k, v in model.state_dict().items()},
        "step": int(step),
        "epoch": int(epoch),
        "rng_cpu": torch.get_rng_state(),
    }
    if torch.cuda.is_available():
        state["rng_cuda"] = torch.cuda.get_rng_state()
    if optimizer is not None:
        state["optimizer"] = {"sharded_over": _world()} if sharded else osd
    if extra:
        state["extra"] = extra
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    _atomic_save(state, path)
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
    return path


def load_checkpoint(path: str, model: torch.nn.Module, optimizer=None, map_location=None) -> Dict[str, Any]:
    state = torch.load(path, map_location=map_location or "cpu", weights_only=True)
    model.load_state_dict(state["model"])
    if optimizer is not None and "optimizer" in state:
        osd = state["optimizer"]
        if isinstance(osd, dict) and "sharded_over" in osd:
            if osd["sharded_over"] != _world():
                raise ValueError(f"checkpoint optimizer is sharded over {osd['sharded_over']} ranks, "
                                 f"this job has {_world()}")
            osd = torch.load(optim_shard_path(path, _rank(), _world()), map_location=map_location or "cpu",
                             weights_only=True)
        optimizer.load_state_dict(osd)
    if "rng_cpu" in state:
        torch.set_rng_state(state["rng_cpu"])
    if "rng_cuda" in state and torch.cuda.is_available():
        torch.cuda.set_rng_state(state["rng_cuda"].cpu() if hasattr(state["rng_cuda"], "cpu") else state["rng_cuda"])
    return {"step": state.get("step", 0), "epoch": state.get("epoch", 0), "extra": state.get("extra")}
