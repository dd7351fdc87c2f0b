"""Hardware queues per process (``GPU_MAX_HW_QUEUES``), sized for the engine's streams.

HIP maps every stream of a process round-robin onto ``GPU_MAX_HW_QUEUES`` hardware (AQL) queues,
4 by default.  A training rank of this framework runs at least four streams -- the compute
stream, the weight-gradient side stream (``ops.functional.WgradStream``), the process group's
comm stream, and RCCL's internal streams -- so with 4 queues two of them share one in-order
queue: a comm-stream barrier packet waiting on the side stream's ready event then blocks the
kernels queued behind it on the same hardware queue.  Measured on one MI355X, ResNet-50 bs256
with a process group (``bench.py --force-comm``): 10.6k img/s at 4 queues, 12.64k at 6 or 8,
12.7k without a process group (``profiles/hw_queues.md``).  That is every N > 1 run.

``ensure(n)`` raises the limit to ``n`` before the HIP runtime starts when each GPU hosts at most
one rank.  Ranks sharing a GPU (multi-rank rehearsals on a small box) get ``SHARED`` queues each
instead: 4 processes x 4 queues already over-subscribed the scheduler
(profiles/multirank_rehearsal.md), so an 8 inherited from a one-rank-per-GPU parent (marked by
``AUTO_MARK``) is dropped.  A value the user set is never touched; ``MI355X_DP_HW_QUEUES=0``
leaves the variable alone.  Must run before the first HIP call of the process; counting
devices does not initialise HIP on this stack.

``check(...)`` is called when an engine is built: a process group plus the weight-gradient stream
on fewer than ``MIN_OK`` queues prints one warning (the 17 % cliff is otherwise silent, e.g. when a
user script touched ``torch.cuda`` before importing the framework).
"""
from __future__ import annotations

import os
import sys

DEFAULT = 8
SHARED = 1
MIN_OK = 6
HIP_DEFAULT = 4
AUTO_MARK = "MI355X_DP_HW_QUEUES_AUTO"

# GPU_MAX_HW_QUEUES as it stood when ensure() found HIP already running (None: ensure() ran first)
_late_value = None
_warned = False


def ranks_per_node() -> int:
    for k in ("LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_SIZE"):
        v = os.environ.get(k)
        if v and v.isdigit():
            return max(1, int(v))
    return 1


def ensure(n: int | None = None) -> int | None:
    """Returns the value set, or None when the variable was left alone."""
    global _late_value
    want = int(os.environ.get("MI355X_DP_HW_QUEUES", str(DEFAULT if n is None else n)))
    if want <= 0:
        return None
    try:
        import torch
        if torch.cuda.is_initialized():
            if _late_value is None:
                _late_value = os.environ.get("GPU_MAX_HW_QUEUES", "")
            return None
        devices = torch.cuda.device_count()
    except Exception:
        return None
    if devices == 0:
        return None
    cur = os.environ.get("GPU_MAX_HW_QUEUES")
    if ranks_per_node() > devices:
        if os.environ.get(AUTO_MARK) == "1":  # inherited from a one-rank-per-GPU parent, not the user's
            os.environ.pop("GPU_MAX_HW_QUEUES", None)
            os.environ.pop(AUTO_MARK, None)
            cur = None
        if cur:
            return None
        os.environ["GPU_MAX_HW_QUEUES"] = str(SHARED)
        os.environ[AUTO_MARK] = "1"
        return SHARED
    if cur and cur.isdigit() and int(cur) >= want:
        return None
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(want, 32))
    os.environ[AUTO_MARK] = "1"  # child processes can tell our setting from a user's
    return min(want, 32)


def effective() -> int:
    """Hardware queues this process's HIP runtime is using (best knowledge: the value in the
    environment when HIP started, if ensure() saw HIP already running; else the current one)."""
    v = _late_value if _late_value is not None else os.environ.get("GPU_MAX_HW_QUEUES", "")
    return int(v) if v and v.isdigit() else HIP_DEFAULT


def check(process_group: bool, side_stream: bool, shared_gpu: bool = False, stream=sys.stderr) -> bool:
    """Warn (once per process) when a process group and the weight-gradient stream run on fewer
    than MIN_OK hardware queues.  Returns True when the warning condition holds."""
    global _warned
    if not (process_group and side_stream) or shared_gpu:
        return False
    q = effective()
    if q >= MIN_OK:
        return False
    if not _warned:
        _warned = True
        print(f"[mi355x_dp] warning: {q} hardware queues per process (GPU_MAX_HW_QUEUES) for a process group "
              f"plus the weight-gradient stream; expect ~17% slower steps (profiles/hw_queues.md).  Import "
              f"mi355x_dp.parallel before the first torch.cuda call, or export GPU_MAX_HW_QUEUES={DEFAULT}.",
              file=stream, flush=True)
    return True
