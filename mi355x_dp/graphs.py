"""HIP-graph capture of a fixed-shape training step ("HIP graphs for the
fixed-shape step" -- the reference's ResNet-18 @ 32x32 / 32 images per GPU is launch-bound:
~200 small kernels per step whose launch overhead exceeds their run time).

``GraphedStep(fn)`` runs ``fn`` (a closure over STATIC device tensors: zero_grad -> forward ->
loss -> backward -> optimizer step) a few times on a side stream, captures one call into a
``torch.cuda.CUDAGraph`` (hipGraph on ROCm) and replays it with a single launch.  Per-step
inputs are written into the static tensors before each replay (e.g. ``augment(..., out=x)``).

Contract (standard graph-capture rules): no host synchronisation inside ``fn``, fixed shapes,
scalars baked at capture time (learning rate, optimizer first-step flag -- capture after at
least one eager step), every tensor ``fn`` reads/writes persists across replays.  Gradient
sync: with one rank there is no collective; with several ranks the process group must
support capture (RCCL via ``ProcessGroupNCCL``), the native reducer's host bookkeeping runs
only during capture and the captured all-reduces replay in the recorded order.
"""
from __future__ import annotations

import contextlib

import torch


@contextlib.contextmanager
def capture_open():
    """Announce an open HIP graph capture to the native library: while any capture is open, no
    lazily grown workspace grows -- on any thread or stream -- so nothing is allocated or
    synchronised outside the graph behind the runtime's back (captures use
    ``capture_error_mode="thread_local"``, which only polices the capturing thread; common.h)."""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    lib = _lib.load(True)
    lib.mi_capture_enter()
    try:
        yield
    finally:
        lib.mi_capture_exit()


class GraphedStep:
    def __init__(self, fn, warmup: int = 2):
        from mi355x_dp.ops.functional import WgradStream
        self.fn = fn
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        # warm-up and capture run single-stream (no weight-gradient / shortcut side streams) and on
        # ONE stream: the native library keys lazily allocated workspaces (split-K partials, tail
        # split, BN finalize counters) by stream, so the warm-up allocates exactly what the
        # captured kernels use -- nothing may be allocated inside the capture
        WgradStream.suspended += 1
        try:
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    fn()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            self.graph = torch.cuda.CUDAGraph()
            with capture_open(), torch.cuda.graph(self.graph, stream=side):
                self.out = fn()
        finally:
            WgradStream.suspended -= 1
        torch.cuda.synchronize()
        self.replays = 0

    def __call__(self):
        self.graph.replay()
        self.replays += 1
        return self.out
