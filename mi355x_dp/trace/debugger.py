"""Observability hook in the spirit of the SageMaker Debugger hook the reference's training
container auto-attaches (log nb2:1267-1522): on the first forward of
the training model it prints the parameter inventory ("Total Trainable Params: N" and one
line per parameter), and it records the scalar training loss every ``save_interval`` steps
into the "losses" collection (JSON lines under ``<out_dir>/collections/losses.jsonl``).

Attach explicitly::

    hook = DebuggerHook(out_dir="/opt/ml/output/tensors")
    hook.register_module(model)
    hook.record_loss(loss)          # or hook.register_loss_backward() to capture loss.backward()

or let a training job attach it: ``TrainingJob`` sets ``MI355X_DP_DEBUGGER=<out_dir>`` and the
compat ``sitecustomize`` calls ``install_from_env()``, which registers a global module forward
hook (first parameterised top-level module wins) and records every scalar ``backward()``.
"""
from __future__ import annotations

import json
import os
import threading
import time

import torch

_installed = None


class DebuggerHook:
    def __init__(self, out_dir: str, save_interval: int = 100, rank: int | None = None):
        self.out_dir = out_dir
        self.save_interval = max(1, int(save_interval))
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.step = 0
        self.module = None
        self._lock = threading.Lock()
        os.makedirs(os.path.join(out_dir, "collections"), exist_ok=True)
        print(f"[mi355x_dp.debugger] Creating hook (collections: losses; save_interval={self.save_interval}; "
              f"out_dir={out_dir})", flush=True)

    # ------------------------------------------------------------- parameters
    def register_module(self, module: torch.nn.Module):
        if self.module is not None:
            return
        self.module = module
        self.first_forward_time = time.time()
        total = 0
        lines = []
        for name, p in module.named_parameters():
            if p.requires_grad:
                total += p.numel()
                lines.append(f"[mi355x_dp.debugger] name:{name} count_params:{p.numel()}")
        if self.rank == 0:
            print("\n".join(lines), flush=True)
            print(f"[mi355x_dp.debugger] Total Trainable Params: {total}", flush=True)
        with open(os.path.join(self.out_dir, "collections", "parameters.json"), "w") as f:
            json.dump({"total_trainable_params": total, "first_forward_time": self.first_forward_time,
                       "params": {n: p.numel() for n, p in module.named_parameters() if p.requires_grad}}, f)

    # ------------------------------------------------------------------ losses
    def record_loss(self, loss):
        with self._lock:
            step = self.step
            self.step += 1
        if step % self.save_interval:
            return
        val = float(loss.detach()) if isinstance(loss, torch.Tensor) else float(loss)
        with open(os.path.join(self.out_dir, "collections", "losses.jsonl"), "a") as f:
            f.write(json.dumps({"step": step, "rank": self.rank, "loss": val, "time": time.time()}) + "\n")

    def register_loss_backward(self):
        """Record every scalar tensor's backward() (the loss) without touching user code."""
        orig = torch.Tensor.backward
        hook = self

        def backward(t, *a, **k):
            if t.dim() == 0 and t.requires_grad:
                hook.record_loss(t)
            return orig(t, *a, **k)

        torch.Tensor.backward = backward
        return self


def install_from_env():
    """Called by the compat sitecustomize inside training jobs (MI355X_DP_DEBUGGER=<out_dir>)."""
    global _installed
    out = os.environ.get("MI355X_DP_DEBUGGER")
    if not out or _installed is not None:
        return _installed
    hook = DebuggerHook(out, save_interval=int(os.environ.get("MI355X_DP_DEBUGGER_INTERVAL", "100")))

    def fwd_hook(module, inputs, output):
        if hook.module is None and any(True for _ in module.parameters()) and not _is_child(module):
            hook.register_module(module)

    torch.nn.modules.module.register_module_forward_hook(fwd_hook)
    hook.register_loss_backward()
    _installed = hook
    return hook


def _is_child(module) -> bool:
    # forward hooks fire inner-first; a module whose class lives in torch.nn (a layer) or that was
    # called from inside another module's forward is not the model itself
    import inspect
    for fr in inspect.stack(0)[2:12]:
        self_obj = fr.frame.f_locals.get("self")
        if isinstance(self_obj, torch.nn.Module) and self_obj is not module:
            return True
    return False
