"""Automatic HIP-graph replay of the forward and backward of a foreign-optimizer engine.

The reference's GPU script (cifar10-distributed-smddp-gpu.py:160-167) trains ResNet-18 on 32x32
images at 32 per GPU: ~150 native kernels per step whose launch cost exceeds their run time.
Through the engine-backed DDP (``engine_ddp.py``) its eager loop left the GPU idle ~70 % of the
time (profiles/reference_unmodified_job.md).  The script itself cannot be changed, so the engine
captures what it owns -- the module's forward and the backward of that forward -- as two graphs
per input signature and replays them; the user's loss, ``loss.backward()`` and stock
``optim.SGD`` run eagerly around them exactly as written:

  ``output = model(data)``   -> copy ``data`` into the static input, replay the forward graph,
                                return a copy of the static output wired to
  ``loss.backward()``        -> ``_Replay.backward``: copy the incoming gradient into the static
                                gradient, replay the backward graph (the kernels accumulate the
                                weight gradients straight into the flat buffer, as eagerly).

Gradient collectives of a replayed backward (``comm_mode``, VERDICT r4 item 3 -- the overlap must
be structural, not a matter of host timing):

* ``capture`` (default whenever every collective can be captured: torch ``nccl`` = RCCL, or the
  native ``smddp`` backend on its RCCL path): the BN-buffer broadcast, every bucket's collective
  (issued by the reducer the moment the bucket's last gradient kernel is captured), the
  end-of-backward join and the 1/world scaling are captured INTO the backward graph.  A collective
  is a branch that forks off the compute stream right after its bucket's gradient kernels and
  joins at the end; HIP replays graph branches concurrently (``tools/graph_branch_probe.py``:
  two forked 0.85 ms spins replay in 0.87 ms), so bucket k's all-reduce runs under the rest of
  the replayed backward with no host involvement at all -- and the host issues no per-bucket
  work per step (the reference loop shape is host-bound).
* ``gates`` (IPC collectives, whose flag epochs are chosen on the host per call and cannot be
  replayed): the graph bumps one flag per bucket right after the bucket's last gradient kernel;
  BEFORE the replay is launched, the engine enqueues per bucket a gate kernel on a high-priority
  gate stream (a different hardware-queue pool than the replaying normal-priority stream, so a
  waiting gate never sits in front of the graph's kernels) followed by that bucket's collective --
  each collective is ordered behind exactly its bucket's kernels, whatever the host does next.
  The end-of-backward callback waits (host) for the last gate and raises if any gate timed out,
  before ``backward()`` returns and before any optimizer step can consume the result.
* ``after``: the Python reducer or a comm hook: every bucket is launched after the replay.

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
``0`` disables.  A forward whose previous graphed forward has not been back-propagated yet runs
eagerly, so the static buffers are never overwritten under a pending backward; the rule follows
program order only (not object liveness), so every rank decides alike.  The capture itself is
agreed on by all ranks (``DataParallel._all_ranks_agree``): if it fails on any rank, every rank
runs eagerly.
"""
from __future__ import annotations

import os

import torch

MODE = os.environ.get("MI355X_DP_ENGINE_GRAPH", "auto")
# how a replayed backward's bucket collectives are issued: auto | capture | gates | after
GRAPH_COMM = os.environ.get("MI355X_DP_GRAPH_COMM", "auto")
# auto mode: inputs up to this many elements per rank are graphed (bs32 x 3 x 32 x 32 = 98k;
# ResNet-50 bs256 @ 224 = 38.5M is overlap-bound and stays eager)
MAX_NUMEL = int(os.environ.get("MI355X_DP_ENGINE_GRAPH_MAX_NUMEL", str(1 << 22)))
AFTER = int(os.environ.get("MI355X_DP_ENGINE_GRAPH_AFTER", "2"))
WARMUP = 2
GATES = os.environ.get("MI355X_DP_GRAPH_GATES", "1") != "0"


def capture_safe(engine) -> bool:
    """can every collective of ``engine``'s process group be captured into a HIP graph?"""
    import torch.distributed as dist
    if not engine.flat.grad.is_cuda:
        return False
    try:
        pg = engine.process_group if engine.process_group is not None else dist.distributed_c10d._get_default_group()
        be = str(dist.get_backend(pg))
    except Exception:
        return False
    if be == "nccl":
        return True
    if be == "smddp":
        from . import comm_paths
        mod = comm_paths._native()
        try:
            return mod is not None and bool(mod.capture_safe(comm_paths.backend_of(pg)))
        except Exception:
            return False
    return False


def _backend(engine) -> str:
    import torch.distributed as dist
    try:
        pg = engine.process_group if engine.process_group is not None else dist.distributed_c10d._get_default_group()
        return str(dist.get_backend(pg))
    except Exception:
        return ""


def gates_stream_high_priority(engine) -> bool:
    """gates are queued BEFORE the replay, so the stream that carries them (and the collectives
    behind them) must never share an in-order hardware queue with the normal-priority stream that
    replays the graph: HIP pools hardware queues per priority, so that stream must be high priority.
    smddp: its comm stream (MI355X_DP_SMDDP_HIPRIO, default high); otherwise the engine's gate stream
    (MI355X_DP_GATE_PRIO, default -1 = high).  torch nccl never qualifies: ProcessGroupNCCL's own
    normal-priority stream would wait on the gate events."""
    be = _backend(engine)
    if be == "nccl":
        return False
    if be == "smddp" and os.environ.get("MI355X_DP_SMDDP_HIPRIO", "1").startswith("0"):
        return False
    return int(os.environ.get("MI355X_DP_GATE_PRIO", "-1")) < 0


def comm_mode(engine) -> str:
    """none | capture | gates | after (module docstring)"""
    if not engine.comm_on:
        return "none"
    if engine.reducer is None or engine._comm_hook is not None:
        return "after"
    want = GRAPH_COMM
    safe = capture_safe(engine)
    if want in ("auto", "capture"):
        if safe:
            return "capture"
        want = "gates"
    if want == "gates" and GATES and gates_stream_high_priority(engine):
        return "gates"
    return "after"


class _Replay(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, x, step):
        if x.data_ptr() != step.static_x.data_ptr():
            step.static_x.copy_(x)
        step.fwd.replay()
        step.gen += 1
        ctx.step = step
        ctx.gen = step.gen
        # a copy, not a view of the static buffer: outputs a script keeps past backward (logits
        # saved for an accuracy count) must not change under the next replay -- stock DDP returns
        # fresh tensors too; the copy is one small kernel next to the ~150 launches saved
        return step.static_out.clone()

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        st = ctx.step
        if ctx.gen != st.gen:
            # a later replay of the forward reused the graph's activations: this output's backward
            # would read another step's tensors -- refuse rather than compute wrong gradients
            raise RuntimeError("mi355x_dp: backward of a graphed forward whose buffers a later replay reused "
                               "(back-propagate each graphed output before the next forward, or set "
                               "MI355X_DP_ENGINE_GRAPH=0)")
        st.static_gout.copy_(g)
        eng = st.engine
        st.pending = False
        if st.comm_mode == "gates":
            # every bucket's gate + collective is enqueued BEFORE the replay: structural ordering
            trace = eng._gate_trace_begin()
            eng._gated_launch(st, st.replays + 1, trace)
            st.bwd.replay()
            st.replays += 1
            if trace is not None:
                trace["end"] = torch.cuda.Event(enable_timing=True)
                trace["end"].record()
            eng._graph_gated = st
        else:
            st.bwd.replay()
            st.replays += 1
            if st.comm_mode == "capture":
                eng._graph_comm_done = True  # the graph ran the collectives, the join and the 1/world
            else:
                eng._graph_backward_ran = True  # "none" / "after": launched at the end of backward
        return None, None, None


# how a gate waits: "cp" -- hipStreamWaitValue32 on signal memory, evaluated by the command processor
# (no wave held on a CU while the replayed backward runs); "kernel" -- a one-wave
# polling kernel with a device-side timeout (mi_flag_gate); "auto": cp where the device supports it
GATE_WAIT = os.environ.get("MI355X_DP_GATE_WAIT", "auto")


class BucketGates:
    """One flag word per gradient bucket of a captured backward (misc.hip ``mi_flag_bump`` /
    ``mi_flag_wait`` or ``mi_flag_gate``): the graph bumps a bucket's flag right after the bucket's
    last gradient kernel; after a replay the engine's gate stream waits, per bucket, until the flag
    reaches the replay count and then launches that bucket's collective -- so bucket k's all-reduce
    runs while the rest of the replayed backward still computes, as in eager mode.  With command-
    processor waits (``cp``) nothing can time out into stale data (a collective simply waits for its
    bucket), so the end of backward needs no host wait on the last gate."""

    TIMEOUT_MS = max(1, int(os.environ.get("MI355X_DP_GATE_TIMEOUT_MS", "60000")))

    def __init__(self, n: int):
        import ctypes
        from mi355x_dp.ops import _lib
        from mi355x_dp.ops import kernels  # noqa: F401
        self._lib = _lib
        lib = _lib.load(True)
        self.n = n
        self.cp = GATE_WAIT == "cp" or (GATE_WAIT == "auto" and bool(lib.mi_wait_value_supported()))
        if self.cp:
            # one 8-byte signal per bucket (hipMallocSignalMemory), kept for the process's life
            self.flags = []
            for _ in range(max(n, 1)):
                p = ctypes.c_void_p()
                _lib.check(lib.mi_signal_alloc(ctypes.byref(p)), "mi_signal_alloc")
                self.flags.append(p.value)
        else:
            p = ctypes.c_void_p()
            _lib.check(lib.mi_flags_alloc(n, ctypes.byref(p)), "mi_flags_alloc")
            self.flags = [p.value + 4 * b for b in range(max(n, 1))]
        if BucketGates._err is None:
            host, dev = ctypes.c_void_p(), ctypes.c_void_p()
            _lib.check(lib.mi_host_word_alloc(ctypes.byref(host), ctypes.byref(dev)), "mi_host_word_alloc")
            BucketGates._err = (ctypes.cast(host, ctypes.POINTER(ctypes.c_int)), dev)

    _err = None

    def _flag(self, b):
        import ctypes
        return ctypes.c_void_p(self.flags[b])

    def bump(self, b: int, stream):
        import ctypes
        self._lib.call("mi_flag_bump", self._flag(b), ctypes.c_void_p(stream.cuda_stream))

    def gate(self, b: int, target: int, stream):
        import ctypes
        if self.cp:
            self._lib.call("mi_flag_wait", self._flag(b), target & 0xFFFFFFFF, ctypes.c_void_p(stream.cuda_stream))
        else:
            self._lib.call("mi_flag_gate", self._flag(b), target & 0xFFFFFFFF, BucketGates._err[1], self.TIMEOUT_MS,
                           ctypes.c_void_p(stream.cuda_stream))

    @staticmethod
    def check():
        if BucketGates._err is not None and BucketGates._err[0][0] != 0:
            raise RuntimeError(f"mi355x_dp: a bucket gate waited {BucketGates.TIMEOUT_MS} ms for its gradients "
                               "(graphed backward did not reach the bucket): the collective ran on stale data")


class CapturedStep:
    """The wrapped module's forward and backward for one input signature, as two HIP graphs."""

    def __init__(self, engine, x: torch.Tensor):
        from mi355x_dp.ops.functional import WgradStream
        self.engine = engine
        self.replays = 0
        self.gen = 0  # forward replays: a backward must belong to the latest one
        # True from a forward replay until its backward ran.  Deterministic (program order, not
        # object liveness), so every rank of an SPMD job takes the same eager / replay decision
        self.pending = False
        self.comm_mode = comm_mode(engine)
        self.gates = BucketGates(len(engine.buckets)) if self.comm_mode == "gates" else None
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
            # thread_local: another thread's runtime calls (the smddp backend's watchdog and torch's
            # ProcessGroupNCCL watchdog poll their collectives' events) must not invalidate this
            # capture -- torch's own recommendation with a live NCCL watchdog.  Workspace growth,
            # the one allocation / synchronisation path of the native library, is held off on every
            # thread and stream while the capture is open (capture_open, common.h).
            from mi355x_dp.graphs import capture_open
            with capture_open(), torch.cuda.graph(self.fwd, pool=pool, stream=s, capture_error_mode="thread_local"):
                out = mod(self.static_x)
            if not isinstance(out, torch.Tensor):
                raise TypeError("graphed forward: the module must return one tensor")
            self.static_gout = torch.empty_like(out)
            if self.comm_mode == "capture":
                # the reducer launches each bucket's collective into the capture as its last
                # gradient kernel is captured; the join and the averaging are captured too
                engine._reset()
                if red is not None:
                    red.enabled = True
                engine.require_backward_grad_sync = True
            with capture_open(), torch.cuda.graph(self.bwd, pool=pool, stream=s, capture_error_mode="thread_local"):
                if self.gates is not None:
                    engine._begin_capture_marks(self.gates, s)
                try:
                    if self.comm_mode == "capture":
                        bw = engine._capture_buffer_broadcast()
                        torch.autograd.backward(out, self.static_gout)
                        engine.finish_gradient_sync(average=True)
                        if bw is not None:
                            bw.wait()
                    else:
                        torch.autograd.backward(out, self.static_gout)
                finally:
                    if self.gates is not None:
                        engine._end_capture_marks()  # buckets no kernel marked: bumped at the end
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
        self.pending = True
        return out

    def busy(self) -> bool:
        """the last replayed forward's backward has not run: its static buffers may still be needed.
        Cleared by that backward, or by a completed eager backward of the same engine (the script
        moved on: a late backward of the old output then raises via the generation check)."""
        return self.pending


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
