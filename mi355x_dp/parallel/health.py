"""Distributed health checks (SURVEY.md §5.2 race detection / §5.3 failure detection).

* ``ReplicaChecker`` -- the reference's visible invariant is that every rank prints the
  identical test loss (replicas bit-identical, nb2:1883-1913).  Every ``every`` steps this
  computes a position-weighted fp64 checksum of the flat parameter buffer (one GPU
  kernel), all-reduces MIN and MAX across ranks and raises ``ReplicaDivergence`` on any
  mismatch -- catching missed / duplicated / mis-ordered gradient buckets.
* ``CollectiveWatchdog`` -- host-side timeout around a blocking collective wait for the
  torch backends (the native smddp backend has its own C++ watchdog that aborts the
  communicator); on timeout it reports the rank and exits non-zero so the launcher tears
  down every rank (abort-on-non-zero-status).
* stream-order checking -- ``DataParallel(check_stream_order=True)`` (or
  MI355X_DP_CHECK_STREAM_ORDER=1) runs every bucket's collective on a copy taken on a side
  stream ordered exactly like the comm stream, and at the end of backward compares its
  checksum with the final local gradient; ``StreamOrderViolation`` names the bucket whose
  gradient was written after its collective had been launched (the race class of a
  grad-ready signal issued before the producing kernel, or a producer on another stream).
"""
from __future__ import annotations

import os
import sys
import threading
import time

import torch
import torch.distributed as dist


class ReplicaDivergence(RuntimeError):
    pass


class StreamOrderViolation(RuntimeError):
    pass


def _dist_on():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


class ReplicaChecker:
    def __init__(self, engine, every: int = 100, group=None):
        self.engine = engine
        self.every = max(1, int(every))
        self.group = group
        self.step = 0
        self.last = None

    def checksum(self) -> float:
        from mi355x_dp.ops import checksum
        if hasattr(self.engine, "wait_param_sync"):
            self.engine.wait_param_sync()  # balanced-shard mode: the parameter all-gathers land first
        v = checksum(self.engine.flat.data)
        return float(v) if not isinstance(v, torch.Tensor) else float(v.item())

    def __call__(self, force: bool = False) -> bool:
        self.step += 1
        if not force and self.step % self.every:
            return True
        c = self.checksum()
        self.last = c
        if not _dist_on():
            return True
        dev = self.engine.flat.data.device
        t = torch.tensor([c, -c], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        hi, lo = float(t[0]), -float(t[1])
        if hi != lo:
            raise ReplicaDivergence(f"rank {dist.get_rank()}: parameter replicas diverged at step {self.step} "
                                    f"(checksum min {lo!r} max {hi!r}, local {c!r})")
        return True


class CollectiveWatchdog:
    """``with CollectiveWatchdog(60, "allreduce bucket 3"): work.wait()``"""

    def __init__(self, timeout_s: float, what: str = "collective"):
        self.timeout_s = timeout_s
        self.what = what
        self._done = threading.Event()

    def _run(self):
        if not self._done.wait(self.timeout_s):
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
            print(f"[mi355x_dp watchdog] rank {rank}: {self.what} did not complete within {self.timeout_s}s; "
                  f"aborting", file=sys.stderr, flush=True)
            os._exit(124)

    def __enter__(self):
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._done.set()
        return False


def check_stream_order(engine) -> list:
    """Violations recorded by an engine built with ``check_stream_order=True``:
    [(bucket, checksum seen by the collective, final checksum)] of the last step."""
    return list(engine.order_violations)
