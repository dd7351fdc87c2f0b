"""Automatic HIP-graph replay of the forward and backward of a foreign-optimizer engine.

The reference's GPU script (cifar10-distributed-smddp-gpu.py:160-167) trains ResNet-18 on 32x32
images at 32 per GPU: ~150 native kernels per step whose launch cost exceeds their run time.
Through the engine-backed DDP (``engine_ddp.py``) its eager loop left the GPU idle ~70 % of the
time (profiles/reference_unmodified_job.md).  The script itself cannot be changed, so the engine
captures what it owns -- the module's forward and the backward of that forward -- as two graphs
per input signature and replays them; the user's loss, ``loss.backward()`` and stock
``optim.SGD`` run eagerly around them exactly as written:

  ``output = model(data)``   -> copy ``data`` into the static input, replay the forward graph,
                                return a detached view of the static output wired to
  ``loss.backward()``        -> ``_Replay.backward``: copy the incoming gradient into the static
                                gradient, replay the backward graph (the kernels accumulate the
                                weight gradients straight into the flat buffer, as eagerly); the
                                engine's end-of-backward callback then launches every bucket's
                                collective (they were not captured) and averages.

Capture (once per signature, after ``AFTER`` eager steps with it): two warm-up passes on the
capture stream size every lazily allocated native workspace for that stream (nothing may be
allocated inside a capture), then the warm-ups' side effects are undone (BN running statistics,
``num_batches_tracked``, the accumulated gradients), then both graphs are captured into one
private memory pool.  Replays are single-stream (no weight-gradient side stream: at this size the
step is launch-bound, not overlap-bound).

Eligibility (else the eager path, unchanged): training mode, grad enabled, one CUDA tensor
argument, gradient sync on (not inside ``no_sync``), no comm hook / stream-order checker / shard
mode, and -- in the default ``auto`` mode -- a small input (``MAX_NUMEL``), since a large step is
not launch-bound and would lose the side-stream overlap.  ``MI355X_DP_ENGINE_GRAPH=1`` forces,
``0`` disables.  A forward whose previous graphed output has not been back-propagated yet (and is
still alive) runs eagerly, so the static buffers are never overwritten under a pending backward.
"""
from __future__ import annotations

import os
import weakref

import torch

MODE = os.environ.get("MI355X_DP_ENGINE_GRAPH", "auto")
# auto mode: inputs up to this many elements per rank are graphed (bs32 x 3 x 32 x 32 = 98k;
# ResNet-50 bs256 @ 224 = 38.5M is overlap-bound and stays eager)
MAX_NUMEL = int(os.environ.get("MI355X_DP_ENGINE_GRAPH_MAX_NUMEL", str(1 << 22)))
AFTER = int(os.environ.get("MI355X_DP_ENGINE_GRAPH_AFTER", "2"))
WARMUP = 2


class _Replay(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, x, step):
        if x.data_ptr() != step.static_x.data_ptr():
            step.static_x.copy_(x)
        step.fwd.replay()
        ctx.step = step
        return step.static_out.detach()

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        st = ctx.step
        st.static_gout.copy_(g)
        st.bwd.replay()
        st.replays += 1
        st.pending = None
        st.engine._graph_backward_ran = True
        return None, None, None


class CapturedStep:
    """The wrapped module's forward and backward for one input signature, as two HIP graphs."""

    def __init__(self, engine, x: torch.Tensor):
        from mi355x_dp.ops.functional import WgradStream
        self.engine = engine
        self.replays = 0
        self.pending = None  # weakref to the last graphed output until its backward ran
        mod = engine.module
        dev = x.device
        self.static_x = torch.empty_strided(tuple(x.shape), tuple(x.stride()), dtype=x.dtype, device=dev)
        self.static_x.copy_(x)
        undo = [engine.buffers.data] + list(engine.buffers.others) + [engine.flat.grad]
        snap = [t.clone() for t in undo]
        s = engine._capture_stream()
        s.wait_stream(torch.cuda.current_stream(dev))
        red = engine.reducer
        old_enabled = red.enabled if red is not None else None
        old_sync = engine.require_backward_grad_sync
        WgradStream.suspended += 1
        try:
            # no bucket bookkeeping / collective may happen inside the warm-ups or the capture
            if red is not None:
                red.enabled = False
            engine.require_backward_grad_sync = False
            with torch.cuda.stream(s):
                for _ in range(WARMUP):
                    out = mod(self.static_x)
                    torch.autograd.backward(out, torch.zeros_like(out))
                del out
                for t, v in zip(undo, snap):
                    t.copy_(v)
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize(dev)
            pool = torch.cuda.graph_pool_handle()
            self.fwd = torch.cuda.CUDAGraph()
            self.bwd = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.fwd, pool=pool, stream=s):
                out = mod(self.static_x)
            if not isinstance(out, torch.Tensor):
                raise TypeError("graphed forward: the module must return one tensor")
            self.static_gout = torch.empty_like(out)
            with torch.cuda.graph(self.bwd, pool=pool, stream=s):
                torch.autograd.backward(out, self.static_gout)
            self.static_out = out.detach()
            del out
        finally:
            WgradStream.suspended -= 1
            if red is not None:
                red.enabled = old_enabled
            engine.require_backward_grad_sync = old_sync
        torch.cuda.synchronize(dev)
        engine._reset()

    def __call__(self, token, x):
        out = _Replay.apply(token, x, self)
        self.pending = weakref.ref(out)
        return out

    def busy(self) -> bool:
        """a graphed output is alive whose backward has not run: its static buffers are in use"""
        return self.pending is not None and self.pending() is not None


def signature(x: torch.Tensor):
    return (tuple(x.shape), tuple(x.stride()), x.dtype, x.device)


def eligible(engine, args, kwargs) -> bool:
    if MODE == "0" or not engine.foreign_optimizer or kwargs or len(args) != 1:
        return False
    x = args[0]
    if not (isinstance(x, torch.Tensor) and x.is_cuda and not x.requires_grad):
        return False
    if MODE != "1" and x.numel() > MAX_NUMEL:
        return False
    if not (engine.module.training and torch.is_grad_enabled() and engine.require_backward_grad_sync):
        return False
    if engine._comm_hook is not None or engine.check_stream_order or engine.sharded:
        return False
    return not torch.cuda.is_current_stream_capturing()


__all__ = ["CapturedStep", "eligible", "signature", "MODE", "MAX_NUMEL", "AFTER"]
