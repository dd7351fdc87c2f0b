"""Per-size collective path selection for the native ``smddp`` backend.

On one xGMI-connected node a gradient all-reduce can take three paths: RCCL's rings, the one-shot
IPC kernel (every rank reads every peer's slot once: one flag round, latency-bound sizes) or the
two-shot IPC kernel (reduce-scatter into the own slot + all-gather: 2/world of the bucket per
point-to-point link).  Which is fastest at which size is a property of the fabric, the RCCL build
and the GPU count -- so it is measured, not assumed:

* ``probe_paths(group)`` times each path per size on the live group (every path forced in turn
  through the backend's ``set_ipc_paths``), MAX over ranks, and returns the table;
* ``choose_paths(rows)`` turns a table into the backend's two thresholds: the largest size up to
  which IPC beats RCCL at every probed size (``threshold_bytes``), and the largest size up to which
  the one-shot beats the two-shot (``oneshot_bytes``).  Pure function, identical on every rank
  because the table is;
* ``apply_paths(group, ...)`` installs them, so each bucket collective the engine issues takes the
  measured-fastest path for its size.

RCCL stays the default until a probe says otherwise (``bench.py`` records the probe table of every
multi-GPU run in its JSON line).
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

RCCL, IPC1, IPC2 = "rccl", "ipc_oneshot", "ipc_twoshot"
BIG = 1 << 62


def _native():
    from . import _smddp_native
    return _smddp_native.load()


def backend_of(group=None):
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    return pg._get_backend(torch.device("cuda"))


def ipc_info(group=None) -> Optional[Dict[str, int]]:
    """the smddp backend's IPC state ({on, cap_bytes, oneshot_bytes, threshold_bytes, flags_*}), or
    None for another backend"""
    mod = _native()
    if mod is None:
        return None
    try:
        return dict(mod.ipc_info(backend_of(group)))
    except Exception:
        return None


def apply_paths(group, threshold_bytes: int, oneshot_bytes: int) -> None:
    _native().set_ipc_paths(backend_of(group), int(threshold_bytes), int(oneshot_bytes))


def choose_paths(rows: Sequence[dict], margin: float = 0.0) -> Tuple[int, int]:
    """``rows``: dicts with ``bytes`` and the ms of each path measured (``rccl``, ``ipc_oneshot``,
    ``ipc_twoshot``; a missing or non-positive entry = not measured).  IPC must beat RCCL by
    ``margin`` (relative) to be chosen.  Returns (threshold_bytes, oneshot_bytes): IPC for every
    size <= threshold (the largest probed size such that IPC won at it and at every smaller probed
    size), one-shot for IPC sizes <= oneshot_bytes (likewise against the two-shot)."""
    rows = sorted(rows, key=lambda r: r["bytes"])

    def t(r, k):
        v = r.get(k)
        return v if v is not None and v > 0 else float("inf")

    threshold = 0
    for r in rows:
        ipc = min(t(r, IPC1), t(r, IPC2))
        if ipc * (1.0 + margin) < t(r, RCCL):
            threshold = r["bytes"]
        else:
            break
    oneshot = 0
    for r in rows:
        if t(r, IPC1) < float("inf") and t(r, IPC1) <= t(r, IPC2):
            oneshot = r["bytes"]
        else:
            break
    return threshold, oneshot


def probe_paths(group=None, device=None, sizes_mb=(0.0625, 0.25, 1.0, 4.0, 16.0, 32.0), iters=5,
                warmup=2) -> List[dict]:
    """Time fp32 all-reduce of each size on each path (MAX over ranks); restores the backend's
    thresholds afterwards.  Needs the smddp backend with IPC enabled (MI355X_DP_SMDDP_IPC=1)."""
    info = ipc_info(group)
    if not info or not info.get("on"):
        raise RuntimeError("probe_paths: the group is not an smddp backend with IPC enabled")
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    world = dist.get_world_size(group)
    buf = torch.zeros(int(max(sizes_mb) * 2**20) // 4, dtype=torch.float32, device=dev)
    old = (info["threshold_bytes"], info["oneshot_bytes"])
    modes = {RCCL: (0, 0), IPC1: (BIG, BIG), IPC2: (BIG, 0)}
    if info.get("only"):  # IPC-only backend: no RCCL communicator to compare against
        del modes[RCCL]
    out = []
    try:
        for mb in sizes_mb:
            n = max(world * 4, (int(mb * 2**20) // 4) // (world * 4) * (world * 4))
            t = buf[:n]
            row = {"bytes": n * 4, "mb": round(n * 4 / 2**20, 4)}
            for name, (thr, one) in modes.items():
                apply_paths(group, thr, one)
                for _ in range(warmup):
                    dist.all_reduce(t, group=group)
                torch.cuda.synchronize(dev)
                dist.barrier(group=group)
                t0 = time.perf_counter()
                for _ in range(iters):
                    dist.all_reduce(t, group=group)
                torch.cuda.synchronize(dev)
                row[name] = (time.perf_counter() - t0) / iters * 1e3
            out.append(row)
    finally:
        apply_paths(group, *old)
    v = torch.tensor([[r.get(k, -1.0) for k in (RCCL, IPC1, IPC2)] for r in out], dtype=torch.float64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MAX, group=group)
    for r, vals in zip(out, v.tolist()):
        for k, x in zip((RCCL, IPC1, IPC2), vals):
            r[k] = round(x, 4)
    return out


def probe_on_new_group(device=None, slot_mb: float = 32.0, **kw) -> dict:
    """bench.py's post-timing probe on a job that runs another backend: a second process group on
    the native smddp backend with IPC enabled (slots of ``slot_mb``), its path table and the
    thresholds it implies, plus the IPC flag memory kind.  Collective over the default group."""
    import os
    from .smddp import register
    register()
    saved = {k: os.environ.get(k) for k in ("MI355X_DP_SMDDP_IPC", "MI355X_DP_SMDDP_IPC_MB")}
    os.environ["MI355X_DP_SMDDP_IPC"] = "1"
    os.environ["MI355X_DP_SMDDP_IPC_MB"] = str(slot_mb)
    try:
        g = dist.new_group(backend="smddp")
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    info = ipc_info(g) or {}
    rows = probe_paths(g, device, **kw)
    thr, one = choose_paths(rows)
    dist.destroy_process_group(g)
    return {"rows": rows, "threshold_bytes": thr, "oneshot_bytes": one,
            "flags": "uncached" if info.get("flags_uncached") else "finegrained" if info.get("flags_finegrained")
            else "coarse"}


def calibrate(group=None, device=None, **kw) -> dict:
    """probe + choose + apply; returns {"rows": table, "threshold_bytes": .., "oneshot_bytes": ..}"""
    rows = probe_paths(group, device, **kw)
    thr, one = choose_paths(rows)
    apply_paths(group, thr, one)
    return {"rows": rows, "threshold_bytes": thr, "oneshot_bytes": one}
