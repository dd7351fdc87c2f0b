"""Hardware queues per process (``GPU_MAX_HW_QUEUES``), sized for the engine's streams.

HIP maps every stream of a process round-robin onto ``GPU_MAX_HW_QUEUES`` hardware (AQL) queues,
4 by default.  A training rank of this framework runs at least four streams -- the compute
stream, the weight-gradient side stream (``ops.functional.WgradStream``), the process group's
comm stream, and RCCL's internal streams -- so with 4 queues two of them share one in-order
queue: a comm-stream barrier packet waiting on the side stream's ready event then blocks the
kernels queued behind it on the same hardware queue.  Measured on one MI355X, ResNet-50 bs256
with a process group (``bench.py --force-comm``): 10.6k img/s at 4 queues, 12.64k at 6 or 8,
12.7k without a process group (``profiles/hw_queues.md``).  That is every N > 1 run.

``ensure(n)`` raises the limit to ``n`` before the HIP runtime starts, but only when each GPU
hosts at most one rank: ranks sharing a GPU keep few queues (4 processes x 4 queues already
over-subscribed the scheduler, profiles/multirank_rehearsal.md).  ``MI355X_DP_HW_QUEUES=0``
leaves the variable alone.  Must run before the first HIP call of the process; counting
devices does not initialise HIP on this stack.
"""
from __future__ import annotations

import os

DEFAULT = 8


def ranks_per_node() -> int:
    for k in ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE"):
        v = os.environ.get(k)
        if v and v.isdigit():
            return max(1, int(v))
    return 1


def ensure(n: int | None = None) -> int | None:
    """Returns the value set, or None when the variable was left alone."""
    want = int(os.environ.get("MI355X_DP_HW_QUEUES", str(DEFAULT if n is None else n)))
    if want <= 0:
        return None
    try:
        import torch
        if torch.cuda.is_initialized():
            return None
        devices = torch.cuda.device_count()
    except Exception:
        return None
    if devices == 0 or ranks_per_node() > devices:
        return None
    cur = os.environ.get("GPU_MAX_HW_QUEUES")
    if cur and cur.isdigit() and int(cur) >= want:
        return None
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(want, 32))
    os.environ[AUTO_MARK] = "1"  # child processes can tell our setting from a user's
    return min(want, 32)


AUTO_MARK = "MI355X_DP_HW_QUEUES_AUTO"
