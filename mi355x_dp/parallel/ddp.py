"""Bucketed data-parallel engine (the MI355X counterpart of torch DDP's Reducer
plus SMDDP's fused gradient buffer, reference gpu.py:148 / SURVEY.md §2.2 C25, §3.2).

Design (MI355X-first):
  * gradients live in ONE flat fp32 buffer (``FlatParams``); buckets are
    contiguous slices of it in backward order -> no copy-in/copy-out kernels.
  * backward kernels signal "grad ready" per parameter; a bucket is launched
    (async all-reduce SUM on its slice, RCCL stream) as soon as all of its
    parameters are ready and every earlier bucket has been launched -- so all
    ranks issue collectives in the same order and the RCCL stream overlaps the
    rest of backward on the compute stream.
  * bucket sizes are chosen for xGMI by the native reducer's link-aware planner
    (csrc/ddp/reducer.cpp): a small first bucket (starts comm early), a small LAST
    bucket (its all-reduce is the exposed tail), and middle buckets sized from an
    alpha-beta model of a ring all-reduce over 7 x 153 GB/s links so per-collective
    latency stays <= ~10 % (``bucket_cap_mb`` / MI355X_DP_BUCKET_MB override it).
  * bucket bookkeeping and in-order launch run in the C++ ``Reducer`` (the
    counterpart of DDP's C++ Reducer); a pure-Python twin is
    kept for builds without the extension (MI355X_DP_PY_REDUCER=1 forces it).
  * averaging (1/world) is folded into the fused optimizer kernel
    (``grad_scale``) instead of a separate scaling pass; ``average=True`` in
    ``finish_gradient_sync`` scales explicitly for foreign optimizers.
  * ``state_dict`` keys carry the ``module.`` prefix exactly like torch DDP so
    checkpoints match the reference's rank-0 ``torch.save`` layout.
  * ``shard_optimizer=True`` is SMDDP's balanced-shard scheme (SURVEY.md §2.4 "SMDDP fused
    balanced shards", §5.8): every bucket is reduce-scattered instead of all-reduced, so rank r
    holds the summed gradient of the r-th 1/world of each bucket; ``FlatSGD`` updates only those
    shards (its momentum buffer holds only them: 1/world of the optimizer state per GPU), and the
    updated parameter shards are all-gathered in place, one collective per bucket, behind the
    optimizer on the comm stream.  The next forward waits for them (a stream wait, no host sync)
    and refreshes the bf16 compute copy.  Same bytes on the wire as the all-reduce (RS + AG), 1/world
    of the optimizer work and state.  Gradients outside the own shards are undefined after the
    sync, so only ``FlatSGD`` can drive this mode.
"""
from __future__ import annotations

import contextlib
import functools
import os
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .flat import FlatBuffers, FlatParams

_ENV_BUCKET_MB = os.environ.get("MI355X_DP_BUCKET_MB")
DEFAULT_BUCKET_MB = float(_ENV_BUCKET_MB) if _ENV_BUCKET_MB else None  # None: link-aware planner
DEFAULT_FIRST_BUCKET_MB = float(os.environ.get("MI355X_DP_FIRST_BUCKET_MB", "2"))
DEFAULT_LAST_BUCKET_MB = float(os.environ.get("MI355X_DP_LAST_BUCKET_MB", "4"))
# buckets below this are merged into a neighbour (a 4 KB fc.bias bucket is a latency-only collective)
DEFAULT_MIN_BUCKET_MB = float(os.environ.get("MI355X_DP_MIN_BUCKET_MB", "1"))
# issue every bucket collective even at world size 1 (exercises the comm stream / overlap on one GPU)
FORCE_COMM = os.environ.get("MI355X_DP_FORCE_COMM", "0") == "1"
# debug: stage each bucket through a copy taken where its collective starts, and check at the end
# of backward that no gradient was written after its bucket was launched (parallel/health.py)
CHECK_STREAM_ORDER = os.environ.get("MI355X_DP_CHECK_STREAM_ORDER", "0") == "1"
# dtype of the gradient exchange: "fp32" (default) or "bf16" (half the bytes on the wire; the sums
# are rounded to bf16 once, identically on every rank, then cast back into the fp32 gradient)
GRAD_COMM = os.environ.get("MI355X_DP_GRAD_COMM", "fp32")
# measure the all-reduce alpha-beta model on the actual fabric at construction (world > 1, planner
# cap not given explicitly) instead of assuming 7 x 153 GB/s xGMI rings with a 25 us launch cost
CALIBRATE = os.environ.get("MI355X_DP_CALIBRATE", "0") == "1"
# run weight gradients on a side HIP stream, overlapping the data-gradient chain
# (mi355x_dp.ops.functional.WgradStream); CUDA engines only.  "auto" (default): on for models with
# BatchNorm -- their BatchNorm / elementwise-heavy data-gradient chain leaves CUs the weight
# gradients fill (ResNet-152 bs256: 5,580 vs 5,132 img/s) -- and off for GEMM-bound models without
# BatchNorm (a transformer's patch-embedding conv aside), where both streams are MFMA-bound and only
# contend (ViT-B/16 bs256: 6,780 vs 6,435 img/s; profiles/raw/r4_vws*, r4_r152ws0).
# MI355X_DP_WGRAD_STREAM=1 / 0 forces it.
_WS = os.environ.get("MI355X_DP_WGRAD_STREAM", "auto")
WGRAD_STREAM = "auto" if _WS == "auto" else _WS == "1"


def _wgrad_stream_auto(module: nn.Module) -> bool:
    """side stream for conv + BatchNorm networks (the memory-bound BN passes leave CUs to fill)"""
    return any(isinstance(m, nn.modules.batchnorm._BatchNorm) for m in module.modules())
# balanced-shard mode: reduce-scatter gradients, shard-local optimizer, all-gather parameters
SHARD_OPTIMIZER = os.environ.get("MI355X_DP_SHARD_OPTIMIZER", "0") == "1"


def plan_buckets(sizes_bytes: List[int], cap_bytes: int, first_cap_bytes: int, last_cap_bytes: int = None,
                 min_bytes: int = 0) -> List[List[int]]:
    """Greedy contiguous bucketing of tensors (given in backward order); Python twin of the
    native planner (csrc/ddp/reducer.cpp plan_buckets): first bucket capped at
    ``first_cap_bytes``, a tail bucket of at most ``last_cap_bytes`` (planned from the end), the
    rest at ``cap_bytes``; then any bucket below ``min_bytes`` is merged into a neighbour."""
    n = len(sizes_bytes)
    if n == 0:
        return []
    last = cap_bytes if last_cap_bytes is None else last_cap_bytes
    tail_begin, acc = n - 1, sizes_bytes[-1]
    while tail_begin > 0 and acc + sizes_bytes[tail_begin - 1] <= last:
        tail_begin -= 1
        acc += sizes_bytes[tail_begin]
    buckets, cur, cur_bytes = [], [], 0
    cap = first_cap_bytes
    for i in range(tail_begin):
        b = sizes_bytes[i]
        if cur and cur_bytes + b > cap and cur_bytes >= min_bytes:
            buckets.append(cur)
            cur, cur_bytes = [], 0
            cap = cap_bytes
        cur.append(i)
        cur_bytes += b
    if cur:
        buckets.append(cur)
    buckets.append(list(range(tail_begin, n)))
    return merge_small_buckets(buckets, sizes_bytes, min_bytes)


def calibrate_allreduce(process_group=None, device=None, sizes_mb=(0.25, 4.0, 32.0), iters=5, warmup=2):
    """Fit T(S) = alpha + S / B (one all-reduce of S bytes of fp32) on the live process group:
    a few timed all-reduces per size, least squares over sizes, then the MAX of each parameter
    over ranks (every rank must plan the same buckets).  Returns (alpha_us, B_GBps)."""
    import time
    dev = device if device is not None else torch.device("cpu")
    cuda = dev.type == "cuda"
    buf = torch.zeros(int(max(sizes_mb) * 2**20) // 4, dtype=torch.float32, device=dev)
    xs, ys = [], []
    for mb in sizes_mb:
        t = buf[:int(mb * 2**20) // 4]
        for _ in range(warmup):
            dist.all_reduce(t, group=process_group)
        if cuda:
            torch.cuda.synchronize(dev)
        dist.barrier(group=process_group)
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(t, group=process_group)
        if cuda:
            torch.cuda.synchronize(dev)
        xs.append(t.numel() * 4.0)
        ys.append((time.perf_counter() - t0) / iters)
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx if sxx > 0 else 0.0
    slope = max(slope, 1e-15)
    alpha = max(my - slope * mx, 1e-6)
    # worst rank: largest latency and largest per-byte time
    v = torch.tensor([alpha, slope], dtype=torch.float64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MAX, group=process_group)
    alpha, slope = float(v[0]), float(v[1])
    return alpha * 1e6, 1.0 / slope / 1e9


def probe_collectives(process_group=None, device=None, sizes_mb=(0.25, 4.0, 32.0, 128.0), iters=5, warmup=2):
    """Measured collective times on the live group (fp32): all-reduce per size, and at each size
    >= 4 MB reduce-scatter + all-gather (the balanced-shard pair) and a bf16 all-reduce of the same
    element count (grad_comm='bf16'); ms per call and
    ring bus bandwidth 2 (W-1)/W * S / t.  MAX over ranks.  Used by bench.py after its timed region
    so every multi-GPU run records the fabric it ran on."""
    import time
    dev = device if device is not None else torch.device("cpu")
    cuda = dev.type == "cuda"
    world = dist.get_world_size(process_group)
    rank = dist.get_rank(process_group)
    buf = torch.zeros(int(max(sizes_mb) * 2**20) // 4, dtype=torch.float32, device=dev)
    buf16 = torch.zeros(buf.numel(), dtype=torch.bfloat16, device=dev)

    def timed(fn):
        for _ in range(warmup):
            fn()
        if cuda:
            torch.cuda.synchronize(dev)
        dist.barrier(group=process_group)
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        if cuda:
            torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / iters

    rows = []
    for mb in sizes_mb:
        n = (int(mb * 2**20) // 4) // (world * 64) * (world * 64)
        t = buf[:n]
        ar = timed(lambda: dist.all_reduce(t, group=process_group))
        rsag = ar16 = None
        if mb >= 4:
            c = n // world
            mine = t[rank * c:(rank + 1) * c]
            rsag = timed(lambda: (dist.reduce_scatter_tensor(mine, t, group=process_group),
                                  dist.all_gather_into_tensor(t, mine, group=process_group)))
            t16 = buf16[:n]
            ar16 = timed(lambda: dist.all_reduce(t16, group=process_group))  # grad_comm='bf16'
        rows.append([mb, ar, rsag if rsag is not None else -1.0, ar16 if ar16 is not None else -1.0])
    v = torch.tensor(rows, dtype=torch.float64, device=dev)
    dist.all_reduce(v, op=dist.ReduceOp.MAX, group=process_group)
    out = []
    for mb, ar, rsag, ar16 in v.tolist():
        nbytes = mb * 2**20
        row = {"mb": mb, "allreduce_ms": round(ar * 1e3, 4),
               "allreduce_busbw_GBps": round(2 * (world - 1) / world * nbytes / ar / 1e9, 3)}
        if rsag > 0:
            row["rs_plus_ag_ms"] = round(rsag * 1e3, 4)
        if ar16 > 0:
            row["allreduce_bf16_same_elems_ms"] = round(ar16 * 1e3, 4)
        out.append(row)
    return out


def calibrated_cap(alpha_us, bw_gbps, overhead=0.1, min_bytes=4 << 20, max_bytes=64 << 20):
    """bucket size whose all-reduce spends `overhead` of its time in the fixed latency alpha"""
    s = alpha_us * 1e-6 * (1.0 - overhead) / overhead * bw_gbps * 1e9
    return int(max(min_bytes, min(max_bytes, s)))


def merge_small_buckets(buckets: List[List[int]], sizes_bytes: List[int], min_bytes: int) -> List[List[int]]:
    """Merge every bucket smaller than ``min_bytes`` into its successor (the last one into its
    predecessor), so no collective is issued for a latency-only sliver."""
    out = [list(b) for b in buckets]
    size = lambda b: sum(sizes_bytes[i] for i in b)  # noqa: E731
    i = 0
    while len(out) > 1 and i < len(out):
        if size(out[i]) >= min_bytes:
            i += 1
            continue
        if i + 1 < len(out):
            out[i + 1] = out[i] + out[i + 1]
            del out[i]
        else:
            out[i - 1] = out[i - 1] + out[i]
            del out[i]
    return out


class DataParallel(nn.Module):
    """Synchronous data parallelism over a flat gradient buffer.

    Usage::

        model = DataParallel(resnet50().cuda())
        opt = FlatSGD(model, lr=0.1, momentum=0.9)
        loss = F.cross_entropy(model(x), y); loss.backward(); opt.step(); opt.zero_grad()
    """

    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: Optional[float] = DEFAULT_BUCKET_MB,
                 first_bucket_mb: float = DEFAULT_FIRST_BUCKET_MB, broadcast_buffers: bool = True,
                 bf16_copy: Optional[bool] = None, last_bucket_mb: float = DEFAULT_LAST_BUCKET_MB,
                 min_bucket_mb: float = DEFAULT_MIN_BUCKET_MB, force_comm: bool = FORCE_COMM,
                 check_stream_order: bool = CHECK_STREAM_ORDER, grad_comm: str = GRAD_COMM,
                 wgrad_stream=WGRAD_STREAM, calibrate: bool = CALIBRATE,
                 shard_optimizer: bool = SHARD_OPTIMIZER, device_ids=None, output_device=None, dim: int = 0,
                 find_unused_parameters: bool = False, gradient_as_bucket_view: bool = True,
                 static_graph: bool = False, foreign_optimizer: bool = False):
        """The trailing keyword arguments are torch DDP's (and SMDDP v1's), accepted so the
        engine is a drop-in ``DistributedDataParallel``: ``device_ids`` / ``output_device`` must
        name the module's own device (one process per GPU), ``dim`` must be 0 (batch-dim data
        parallelism); ``find_unused_parameters`` is implied (a bucket whose parameters got no
        gradient is still reduced at the end of backward), gradients are always bucket views, and
        ``static_graph`` needs no special path (the bucket order is fixed).

        ``foreign_optimizer=True`` is torch DDP's contract for an optimizer the engine does not own
        (stock ``optim.SGD`` over ``engine.parameters()``, what the reference scripts use,
        gpu.py:156-158): gradients are averaged over the ranks when ``backward()`` returns (a final
        autograd callback joins the bucket collectives and scales by 1/world); a ``zero_grad`` that
        set the gradients to None re-points them at the flat buffer (zeroed) at the next forward;
        and parameters changed in place since the last forward refresh the bf16 compute copy and
        the transposed data-gradient operands first.  Shard mode needs FlatSGD, so it is refused."""
        super().__init__()
        if dim != 0:
            raise ValueError("DataParallel: only batch-dimension (dim=0) data parallelism")
        mod_dev = next((p.device for p in module.parameters()), None)
        for d in list(device_ids or []) + ([output_device] if output_device is not None else []):
            d = torch.device("cuda", d) if isinstance(d, int) else torch.device(d)
            if mod_dev is not None and d.type == "cuda" and mod_dev.type == "cuda" and \
                    d.index not in (None, mod_dev.index):
                raise ValueError(f"DataParallel: device {d} is not the module's device {mod_dev} "
                                 "(one process per GPU)")
        if foreign_optimizer and shard_optimizer:
            raise ValueError("DataParallel: shard_optimizer=True needs FlatSGD (foreign_optimizer=True refused)")
        self.foreign_optimizer = bool(foreign_optimizer)
        self._final_cb_pending = False
        self.require_backward_grad_sync = True
        self.module = module
        self.process_group = process_group
        self.distributed = dist.is_available() and dist.is_initialized()
        self.world_size = dist.get_world_size(process_group) if self.distributed else 1
        self.rank = dist.get_rank(process_group) if self.distributed else 0
        self.broadcast_buffers = broadcast_buffers and self.distributed and self.world_size > 1
        # collectives are issued when there is a peer -- or at world 1 when forced (trace / overlap runs)
        self.comm_on = self.distributed and (self.world_size > 1 or force_comm)
        self.check_stream_order = bool(check_stream_order)
        self.order_violations = []
        self._buf_works = []

        params = [p for p in module.parameters() if p.requires_grad]
        params = list(reversed(params))  # approximate backward order
        from mi355x_dp.models.layers import Conv2d as _NativeConv
        # conv weights in the native kernels' [K][R][S][C] layout -- only where those kernels run (on
        # host tensors the stock convolutions then see torch's own layout and round identically)
        on_gpu = any(p.is_cuda for p in params)
        kernel_ids = {id(m.weight) for m in module.modules() if isinstance(m, _NativeConv)} if on_gpu else set()
        self.buffers = FlatBuffers(list(module.buffers()))
        if bf16_copy is None:  # the bf16 compute shadow serves the bf16 kernels only
            from mi355x_dp.ops.fp32 import COMPUTE_FP32
            bf16_copy = not COMPUTE_FP32

        from . import _reducer_native
        native = _reducer_native.load()
        sizes = [p.numel() * 4 for p in params]
        self.calibration = None
        if bucket_cap_mb is None and calibrate and self.distributed and self.world_size > 1:
            dev = params[0].device if params else torch.device("cpu")
            a_us, bw = calibrate_allreduce(process_group, dev)
            cap = calibrated_cap(a_us, bw)
            self.calibration = {"alpha_us": round(a_us, 2), "algbw_GBps": round(bw, 2), "cap_mb": round(cap / 2**20, 2)}
        elif bucket_cap_mb is None:
            cap = (native.link_aware_cap(self.world_size) if native is not None
                   else int(32 * 2**20))
        else:
            cap = int(bucket_cap_mb * 2**20)
        self.bucket_cap_bytes = cap
        first_b, last_b = int(first_bucket_mb * 2**20), min(cap, int(last_bucket_mb * 2**20))
        min_b = int(min_bucket_mb * 2**20)
        if native is not None:
            self.buckets = [list(b) for b in native.plan_buckets(sizes, cap, first_b, last_b, min_b)]
        else:
            self.buckets = plan_buckets(sizes, cap, first_b, last_b, min_b)
        # balanced shards: every bucket padded to world x 64 elements (equal, aligned shards)
        self.sharded = bool(shard_optimizer)
        self.bucket_align = 64 * (self.world_size if self.sharded else 1)
        self.flat = FlatParams(params, bf16_copy=bf16_copy, kernel_layout_ids=kernel_ids,
                               group_ends=[b[-1] for b in self.buckets] if self.sharded else (),
                               group_align=self.bucket_align)
        self.bucket_of = {}
        for b, idxs in enumerate(self.buckets):
            for i in idxs:
                self.bucket_of[i] = b
        self.bucket_ranges = []
        for idxs in self.buckets:
            lo = self.flat.offsets[idxs[0]]
            hi = self.flat.offsets[idxs[-1]] + self.flat.params[idxs[-1]].numel()
            hi = min(self.flat.numel, (hi + self.bucket_align - 1) // self.bucket_align * self.bucket_align)
            self.bucket_ranges.append((lo, hi))
        # this rank's [lo, hi) of every bucket (the whole bucket unless sharded)
        self.shard_ranges = []
        for lo, hi in self.bucket_ranges:
            if self.sharded:
                c = (hi - lo) // self.world_size
                self.shard_ranges.append((lo + self.rank * c, lo + (self.rank + 1) * c))
            else:
                self.shard_ranges.append((lo, hi))
        self._gather_works = []
        self._gather_pending = False
        self._pending = [0] * len(self.buckets)
        self._ready = [False] * len(self.buckets)
        self._works = []
        self._next = 0
        self._param_ready = [False] * len(self.flat.params)
        self._py_comm_calls = 0

        self.reducer = None
        self._capture_marks = None  # graph capture of a backward: bucket-gate bookkeeping
        self._staging = {}
        if grad_comm not in ("fp32", "bf16"):
            raise ValueError(f"grad_comm must be 'fp32' or 'bf16', not {grad_comm!r}")
        self.grad_comm = grad_comm
        self._comm_buf = (torch.empty(self.flat.grad.numel(), dtype=torch.bfloat16, device=self.flat.grad.device)
                          if grad_comm == "bf16" and self.comm_on and not self.check_stream_order else None)
        self._sent = set()
        if native is not None and not self.check_stream_order:
            pg = None
            if self.comm_on:
                pg = process_group if process_group is not None else dist.distributed_c10d._get_default_group()
            self.reducer = native.Reducer(self.flat.grad, [int(o) for o in self.flat.offsets],
                                          [p.numel() for p in self.flat.params], self.buckets, pg, self.bucket_align,
                                          bool(force_comm), self._comm_buf, self.sharded)
        self._comm_hook = None
        self.wgrad_stream = None
        if wgrad_stream == "auto":
            wgrad_stream = _wgrad_stream_auto(module)
        if wgrad_stream and self.flat.grad.is_cuda:
            from mi355x_dp.ops.functional import WgradStream
            self.wgrad_stream = WgradStream(self.flat.grad.device)
            from mi355x_dp.utils import hwqueues
            self.hw_queue_warning = hwqueues.check(
                self.comm_on, True, shared_gpu=hwqueues.ranks_per_node() > torch.cuda.device_count())
        for i, p in enumerate(self.flat.params):
            cb = functools.partial(self._ready_native, i) if self.reducer is not None \
                else self._make_ready_cb(i)
            p._mi_on_grad_ready = cb
            p._mi_side = self.wgrad_stream
            hook_cb = functools.partial(self.wgrad_stream.mark, cb) if self.wgrad_stream is not None else cb
            p.register_post_accumulate_grad_hook(self._make_hook(i, hook_cb))

        if self.distributed and self.world_size > 1:
            # one broadcast of the whole flat parameter buffer (+ buffers) from rank 0
            dist.broadcast(self.flat.data, 0, group=process_group)
            if self.buffers.buffers:
                dist.broadcast(self.buffers.data, 0, group=process_group)
            self.flat.refresh_bf16()
        # a state_dict loaded into the wrapped model (checkpoint resume) writes the fp32 masters in
        # place; the bf16 compute copy and the transposed dgrad copies follow it
        module.register_load_state_dict_post_hook(lambda _m, _keys: self.flat.refresh_bf16())
        self._params_version = self.flat.params_version()
        self._params_dirty = False
        if self.foreign_optimizer:
            _watch_optimizer_steps(self)
        self._reset()

    @property
    def bucket_trace(self):
        """(bucket, bytes, launch_us) of the last step, launch time relative to forward start
        (native reducer only): the order and timing in which buckets went to the comm stream."""
        return list(self.reducer.trace) if self.reducer is not None else []

    @property
    def comm_calls(self) -> int:
        if self.reducer is not None and self._comm_hook is None:
            return self.reducer.comm_calls
        return self._py_comm_calls

    @property
    def native_reducer(self) -> bool:
        return self.reducer is not None

    # -------------------------------------------------------------- hooks
    def _make_ready_cb(self, i):
        def cb():
            self._mark_ready(i)
        return cb

    @staticmethod
    def _make_hook(i, cb):
        def hook(p):
            cb()
        return hook

    def _ready_native(self, i):
        if self._capture_marks is not None:
            self._capture_mark(i)
            return
        if self._comm_hook is None:
            self.reducer.mark_ready(i)
        else:
            self._mark_ready(i)

    def register_comm_hook(self, state, hook):
        """torch DDP's communication hook: ``hook(state, bucket) -> Future[Tensor]`` replaces the
        bucket all-reduce.  ``bucket`` offers DDP's GradBucket interface (``index``, ``buffer`` --
        the bucket's slice of the flat gradient, ``gradients``, ``parameters``, ``is_last``,
        ``set_buffer``); the future's tensor becomes the bucket's gradient.  As in torch DDP the hook
        owns the averaging (torch's ``allreduce_hook`` / ``fp16_compress_hook`` /
        ``bf16_compress_hook`` divide by the world size), so ``FlatSGD`` no longer scales by
        1/world.  Buckets keep the engine's plan and launch order; the hooked path runs in Python."""
        if self._comm_hook is not None:
            raise RuntimeError("register_comm_hook can only be called once")
        if self.sharded or self.check_stream_order or self.grad_comm != "fp32":
            raise RuntimeError("register_comm_hook: not combinable with shard_optimizer, check_stream_order "
                               "or grad_comm='bf16' (a hook can compress itself)")
        self._comm_hook = (state, hook)
        self._reset()

    def _reset(self):
        if self.reducer is not None:
            self.reducer.reset()
            if self._comm_hook is None:
                return
        for b, idxs in enumerate(self.buckets):
            self._pending[b] = len(idxs)
            self._ready[b] = False
        self._param_ready = [False] * len(self.flat.params)
        self._works = []
        self._sent = set()
        self._next = 0

    @contextlib.contextmanager
    def no_sync(self):
        """torch DDP's gradient-accumulation context: backward passes inside it only accumulate
        into the flat gradient buffer (no collective); the first backward after it reduces the
        accumulated sum.  Not available in balanced-shard mode (non-own shards are not kept)."""
        if self.sharded:
            raise RuntimeError("no_sync() is not supported with shard_optimizer=True")
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        if self.reducer is not None:
            self.reducer.enabled = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old
            if self.reducer is not None:
                self.reducer.enabled = old

    def _mark_ready(self, i):
        if self._capture_marks is not None:
            self._capture_mark(i)
            return
        if not self.require_backward_grad_sync:
            return
        if self._param_ready[i]:
            return
        self._param_ready[i] = True
        b = self.bucket_of[i]
        self._pending[b] -= 1
        if self._pending[b] == 0:
            self._ready[b] = True
            self._launch_ready()

    def _launch_ready(self):
        while self._next < len(self.buckets) and self._ready[self._next]:
            self._launch(self._next)
            self._next += 1

    def _launch(self, b):
        lo, hi = self.bucket_ranges[b]
        if self.check_stream_order:
            self._launch_checked(b, lo, hi)
            return
        if not self.comm_on:
            return
        if self._comm_hook is not None:
            state, hook = self._comm_hook
            self._works.append((lo, hi, hook(state, _GradBucket(self, b))))
            self._py_comm_calls += 1
            return
        buf = self.flat.grad[lo:hi]
        if self._comm_buf is not None:
            self._comm_buf[lo:hi].copy_(buf)
            buf = self._comm_buf[lo:hi]
            self._sent.add(b)
        if self.sharded:
            c = (hi - lo) // self.world_size
            w = dist.reduce_scatter_tensor(buf[self.rank * c:(self.rank + 1) * c], buf, op=dist.ReduceOp.SUM,
                                           group=self.process_group, async_op=True)
        else:
            w = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.process_group, async_op=True)
        self._works.append(w)
        self._py_comm_calls += 1

    def _launch_checked(self, b, lo, hi):
        """Stream-order check mode: the bucket's collective runs on a copy of its slice taken on
        a side stream that waits for everything the compute stream had enqueued when the bucket
        became ready -- i.e. exactly what the comm stream sees.  finish_gradient_sync compares a
        checksum of that copy with one of the final local gradient; a mismatch means a kernel
        wrote a gradient after its bucket was handed to the collective (grad-ready signalled
        too early, or a producer on an unsynchronised stream)."""
        from mi355x_dp.ops import checksum
        g = self.flat.grad
        if g.is_cuda:
            side = self._staging.get("stream")
            if side is None:
                side = self._staging["stream"] = torch.cuda.Stream(device=g.device)
            side.wait_stream(torch.cuda.current_stream(g.device))
            with torch.cuda.stream(side):
                stage = g[lo:hi].clone()
                seen = checksum(stage)
                w = self._reduce_stage(stage) if self.comm_on else None
        else:
            stage = g[lo:hi].clone()
            seen = checksum(stage)
            w = self._reduce_stage(stage) if self.comm_on else None
        if w is not None:
            self._py_comm_calls += 1
        self._works.append((b, lo, hi, stage, seen, w))

    def _reduce_stage(self, stage):
        if self.sharded:
            c = stage.numel() // self.world_size
            return dist.reduce_scatter_tensor(stage[self.rank * c:(self.rank + 1) * c], stage, op=dist.ReduceOp.SUM,
                                              group=self.process_group, async_op=True)
        return dist.all_reduce(stage, op=dist.ReduceOp.SUM, group=self.process_group, async_op=True)

    def _finish_checked(self):
        from mi355x_dp.ops import checksum
        g = self.flat.grad
        side = self._staging.get("stream")
        if side is not None:
            torch.cuda.current_stream(g.device).wait_stream(side)
        for b, lo, hi, stage, seen, w in self._works:
            final = checksum(g[lo:hi])
            if w is not None:
                w.wait()
            if float(seen) != float(final):
                self.order_violations.append((b, float(seen), float(final)))
            g[lo:hi].copy_(stage)
        self._works = []
        if self.order_violations:
            from .health import StreamOrderViolation
            b, s0, s1 = self.order_violations[0]
            raise StreamOrderViolation(
                f"bucket {b} (params {self.buckets[b]}) changed after its all-reduce was launched: checksum "
                f"seen by the collective {s0!r} != final local gradient {s1!r} ({len(self.order_violations)} "
                f"bucket(s) affected)")

    # ------------------------------------------------------------ public
    def _join_side(self):
        if self.wgrad_stream is not None:
            self.wgrad_stream.join()

    # ------------------------------------------------- balanced-shard mode
    def gather_params(self):
        """Shard mode, after the optimizer updated this rank's shards of ``flat.data``: all-gather
        every bucket's parameter shards in place (async, comm stream).  ``wait_param_sync`` -- called
        by the next forward, ``state_dict`` and ``sync_params`` -- joins them."""
        if not self.sharded:
            return
        self._gather_pending = True
        if not self.comm_on:
            return
        if self.reducer is not None:
            self.reducer.gather_params(self.flat.data)
            return
        for (lo, hi), (slo, shi) in zip(self.bucket_ranges, self.shard_ranges):
            self._gather_works.append(dist.all_gather_into_tensor(self.flat.data[lo:hi], self.flat.data[slo:shi],
                                                                  group=self.process_group, async_op=True))
            self._py_comm_calls += 1

    def wait_param_sync(self):
        """Make the current stream wait for the parameter all-gathers, then refresh the bf16
        compute copy (and the transposed data-gradient operands) from the gathered fp32 masters."""
        if not self._gather_pending:
            return
        if self.reducer is not None:
            self.reducer.wait_gather()
        for w in self._gather_works:
            w.wait()
        self._gather_works = []
        self._gather_pending = False
        self.flat.refresh_bf16()

    def _foreign_prepare(self):
        """foreign_optimizer mode, before a forward: gradients set to None by the user's
        zero_grad are re-pointed at the (zeroed) flat buffer; parameters the user's optimizer
        changed (any optimizer step -- a global step hook -- or any in-place write, seen in the
        parameters' version counters) refresh the bf16 / transposed compute copies."""
        v = self.flat.params_version()
        if v != self._params_version or self._params_dirty:
            self.flat.refresh_bf16()  # + transposed dgrad operands
            self._params_version = v
            self._params_dirty = False
        if torch.is_grad_enabled() and self.flat.reattach_grads():
            self.flat.zero_grad()

    def _final_callback(self):
        self._final_cb_pending = False
        if self.__dict__.pop("_graph_comm_done", False):
            return  # a replayed backward graph already ran its collectives, their join and the 1/world
        graph_ran = self.__dict__.pop("_graph_backward_ran", False)
        if graph_ran and self.comm_on:
            self._mark_all_ready()
        if not graph_ran and "_graph_gated" not in self.__dict__:
            # an eager backward completed: the script moved past any graphed output it never
            # back-propagated, so the graphs may replay again (same program order on every rank)
            for g in self.__dict__.get("_graphs", {}).values():
                g.pending = False
        gated = self.__dict__.pop("_graph_gated", None)
        self.finish_gradient_sync(average=True)
        if gated is not None and not gated.gates.cp:
            # a polling gate that timed out let its collective run on stale gradients: find out (host
            # wait for the last gate, i.e. until the replayed backward reached its last bucket) and
            # raise before backward() returns -- before any optimizer step can use the result.
            # Command-processor gates cannot time out into stale data: no host wait at all
            from .step_graph import BucketGates
            ev = self.__dict__.pop("_last_gate_event", None)
            if ev is not None:
                ev.synchronize()
            BucketGates.check()

    def _arm_final_callback(self, out):
        """torch DDP's end-of-backward contract: the first gradient that reaches this forward's
        output queues an autograd final callback that joins every bucket collective and averages,
        so ``p.grad`` holds the all-reduced mean when ``backward()`` returns."""
        t = out
        while isinstance(t, (tuple, list)) and t:
            t = t[0]
        # a backward that raised after queueing the callback (an OOM the script catches and
        # retries) never ran it: re-arm on every forward so that no later step skips its sync
        self._final_cb_pending = False
        if not (isinstance(t, torch.Tensor) and t.requires_grad):
            return

        def hook(g):
            if not self._final_cb_pending:
                self._final_cb_pending = True
                torch.autograd.Variable._execution_engine.queue_callback(self._final_callback)
            return g
        t.register_hook(hook)

    def forward(self, *args, **kwargs):
        self._join_side()  # a backward whose sync was skipped (no_sync / accumulation) left side work
        if self.foreign_optimizer:
            self._foreign_prepare()
        self._reset()
        self.wait_param_sync()
        self._wait_buffer_sync()
        self._graph_bcast = False
        out = self._graphed_forward(args, kwargs) if self.foreign_optimizer else None
        if out is None:
            out = self.module(*args, **kwargs)
        if self.foreign_optimizer and torch.is_grad_enabled():
            self._arm_final_callback(out)
        if self._graph_bcast:
            pass  # captured into this step's backward graph (step_graph comm_mode "capture")
        elif self.broadcast_buffers and self.buffers.buffers and self.module.training:
            # torch DDP broadcasts rank 0's buffers synchronously BEFORE every training forward
            # (SURVEY.md X4), on the critical path.  Same values, off the critical path: broadcast
            # AFTER this forward's BN kernels (which update the running statistics) are enqueued;
            # the comm stream runs it behind backward, and it is waited for before the next
            # forward -- when every rank again starts from rank 0's buffers.  Backward never
            # touches the buffers, and the broadcast precedes every bucket collective on all ranks.
            self._buf_works.append(dist.broadcast(self.buffers.data, 0, group=self.process_group, async_op=True))
        return out

    # ------------------------------------- foreign optimizer: graphed forward + backward
    def _capture_stream(self):
        s = getattr(self, "_cap_stream", None)
        if s is None:
            s = self._cap_stream = torch.cuda.Stream(device=self.flat.grad.device)
        return s

    def _graphed_forward(self, args, kwargs):
        """Replay of the captured forward (+ its backward at ``loss.backward()``) for a small,
        launch-bound step (parallel/step_graph.py); None: run the module eagerly."""
        from . import step_graph
        if self.__dict__.get("_graph_disabled") or not step_graph.eligible(self, args, kwargs):
            return None
        x = args[0]
        key = step_graph.signature(x)
        graphs = self.__dict__.setdefault("_graphs", {})
        st = graphs.get(key)
        if st is None:
            seen = self.__dict__.setdefault("_graph_seen", {})
            seen[key] = seen.get(key, 0) + 1
            if seen[key] <= step_graph.AFTER:
                return None
            err = None
            try:
                st = step_graph.CapturedStep(self, x)
            except Exception as e:  # never fail a training step over the optimisation: run eagerly
                err, st = e, None
            # rank-symmetric: every rank reaches this capture on the same step (the seen counts and
            # eligibility are SPMD-symmetric), so one MIN all-reduce of the success flag decides for
            # all of them -- a rank whose capture failed must not run eagerly while its peers replay
            # graphs with captured collectives (cifar10-distributed-smddp-gpu.py:148,160-168)
            if not self._all_ranks_agree(err is None):
                import warnings
                self._graph_disabled = True
                why = f"failed here ({err!r})" if err is not None else "failed on another rank"
                warnings.warn(f"mi355x_dp: graph capture of the forward/backward {why}; "
                              "every rank runs this engine eagerly", stacklevel=3)
                return None
            graphs[key] = st
        elif any(g.busy() for g in graphs.values()):
            # deterministic (backward-not-yet-run, not object liveness): the same on every rank
            return None
        tok = self.__dict__.get("_graph_token")
        if tok is None:
            tok = self._graph_token = torch.zeros((), device=x.device, requires_grad=True)
        self._graph_bcast = st.comm_mode == "capture"
        return st(tok, x)

    def _all_ranks_agree(self, ok: bool) -> bool:
        """True iff ``ok`` holds on every rank of the engine's process group (MIN all-reduce of a
        flag, on the engine's device); world 1: ``ok``."""
        if self.world_size <= 1 or not dist.is_initialized():
            return ok
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self.flat.grad.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.process_group)
        return bool(int(flag.item()))

    def _capture_buffer_broadcast(self):
        """inside the capture of a backward graph (comm_mode "capture"): rank 0's BN buffers, as
        updated by the replayed forward, broadcast on the comm stream ahead of the bucket
        collectives (the eager engine issues it after the forward; same values, same order)"""
        if self.broadcast_buffers and self.buffers.buffers and self.module.training:
            return dist.broadcast(self.buffers.data, 0, group=self.process_group, async_op=True)
        return None

    # ------------------------------------- graphed backward: per-bucket gates (step_graph)
    def _begin_capture_marks(self, gates, stream):
        """Inside the capture of a backward: as each bucket's gradients complete (in bucket order,
        like the reducer), capture a bump of that bucket's gate flag on the capture stream."""
        self._capture_marks = {"gates": gates, "stream": stream, "seen": set(), "next": 0,
                               "pending": [len(b) for b in self.buckets]}

    def _capture_mark(self, i):
        cm = self._capture_marks
        if i in cm["seen"]:
            return
        cm["seen"].add(i)
        cm["pending"][self.bucket_of[i]] -= 1
        while cm["next"] < len(self.buckets) and cm["pending"][cm["next"]] == 0:
            cm["gates"].bump(cm["next"], cm["stream"])
            cm["next"] += 1

    def _end_capture_marks(self):
        cm, self._capture_marks = self._capture_marks, None
        for b in range(cm["next"], len(self.buckets)):  # parameters without a gradient kernel
            cm["gates"].bump(b, cm["stream"])

    def _gate_stream(self):
        # HIGH priority: HIP pools hardware queues per priority, so the gate stream never shares an
        # in-order queue with the normal-priority stream that replays the graph -- a gate enqueued
        # before the replay cannot sit in front of the kernels it waits for
        s = getattr(self, "_gate_s", None)
        if s is None:
            s = self._gate_s = torch.cuda.Stream(device=self.flat.grad.device,
                                                 priority=int(os.environ.get("MI355X_DP_GATE_PRIO", "-1")))
        return s

    def _gate_trace_begin(self):
        if os.environ.get("MI355X_DP_GATE_TRACE", "0") != "1":
            return None
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record()
        return {"t0": t0, "gates": [], "end": None}

    def _smddp_comm_stream(self):
        """the native smddp backend's comm stream (a torch ExternalStream), or None"""
        if "_smddp_cs" not in self.__dict__:
            cs = None
            try:
                from . import comm_paths
                mod = comm_paths._native()
                pg = self.process_group if self.process_group is not None else dist.distributed_c10d._get_default_group()
                if mod is not None and str(dist.get_backend(pg)) == "smddp":
                    h = int(mod.comm_stream(comm_paths.backend_of(pg)))
                    cs = torch.cuda.ExternalStream(h, device=self.flat.grad.device)
            except Exception:
                cs = None
            self._smddp_cs = cs
        return self._smddp_cs

    def _gated_launch(self, step, target, trace=None):
        """BEFORE a replay of a captured backward (comm_mode "gates"): per bucket b, in order, a gate
        kernel on the high-priority gate stream that waits until the graph's bump of b reaches
        ``target`` (this replay), then b's collective issued with the gate stream current -- the
        reducer's ready-mark, any bf16 cast and the collective's producer event are all ordered
        behind that gate, i.e. behind exactly b's gradient kernels."""
        from .step_graph import BucketGates
        BucketGates.check()
        # the native smddp backend (the IPC collectives that take this path): gates straight on its
        # comm stream, each collective issued from that stream too -- its producer event, any bf16
        # cast and the collective all follow the gate in one in-order stream, and no second stream
        # can share a hardware queue with it; otherwise the high-priority gate stream
        gs = self._smddp_comm_stream() or self._gate_stream()
        gs.wait_stream(torch.cuda.current_stream(gs.device))  # the previous step's users of the buckets
        with torch.cuda.stream(gs):
            for b, idxs in enumerate(self.buckets):
                step.gates.gate(b, target, gs)
                if trace is not None:
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record(gs)
                    trace["gates"].append(ev)
                for i in idxs:
                    self.reducer.mark_ready(i)
            last = torch.cuda.Event()
            last.record(gs)
        self._last_gate_event = last
        if trace is not None:
            self._last_gate_trace = trace

    def gate_trace_ms(self):
        """(ms at which each bucket's gate opened, ms at which the replayed backward ended), both
        from the replay's start -- the last graphed step, with MI355X_DP_GATE_TRACE=1."""
        tr = getattr(self, "_last_gate_trace", None)
        if tr is None:
            return None
        torch.cuda.synchronize(self.flat.grad.device)
        return [tr["t0"].elapsed_time(e) for e in tr["gates"]], tr["t0"].elapsed_time(tr["end"])

    def _mark_all_ready(self):
        """after a graph replay: the captured backward wrote every gradient; launch the buckets"""
        for i in range(len(self.flat.params)):
            if self.reducer is not None:
                self._ready_native(i)
            else:
                self._mark_ready(i)

    def _wait_buffer_sync(self):
        for w in self._buf_works:
            w.wait()
        self._buf_works = []

    def finish_gradient_sync(self, average: bool = False):
        """Launch any bucket not yet launched (unused params), then wait for all."""
        self._join_side()
        self._wait_buffer_sync()
        if not self.require_backward_grad_sync:
            return  # inside no_sync(): local accumulation only
        if average and self.sharded:
            raise RuntimeError("shard_optimizer=True: gradients outside this rank's shards are not reduced; "
                               "drive the engine with FlatSGD")
        if self._comm_hook is not None:
            for b in range(len(self.buckets)):
                self._ready[b] = True
            self._launch_ready()
            for lo, hi, fut in self._works:
                t = fut.wait()
                t = t[0] if isinstance(t, (list, tuple)) else t
                dst = self.flat.grad[lo:hi]
                if t.data_ptr() != dst.data_ptr():
                    dst.copy_(t.reshape(-1))
            self._works = []
            return  # the hook averaged
        if self.reducer is not None:
            self.reducer.finish()
            if average and self.world_size > 1:
                self.flat.grad.mul_(1.0 / self.world_size)
            return
        for b in range(len(self.buckets)):
            self._ready[b] = True
        self._launch_ready()
        if self.check_stream_order:
            self._finish_checked()
        else:
            for w in self._works:
                w.wait()
            self._works = []
            for b in sorted(self._sent):
                lo, hi = self.shard_ranges[b]
                self.flat.grad[lo:hi].copy_(self._comm_buf[lo:hi])
            self._sent = set()
        if average and self.world_size > 1:
            self.flat.grad.mul_(1.0 / self.world_size)

    @property
    def grad_scale(self) -> float:
        if self.foreign_optimizer:
            return 1.0  # the end-of-backward callback already averaged
        return 1.0 if self._comm_hook is not None and self.comm_on else 1.0 / self.world_size

    def zero_grad(self, set_to_none: bool = False):
        self._join_side()
        self.flat.reattach_grads()
        self.flat.zero_grad()

    def state_dict(self, *args, **kwargs):
        self._wait_buffer_sync()
        self.wait_param_sync()
        return super().state_dict(*args, **kwargs)


_FOREIGN_ENGINES = None


def _watch_optimizer_steps(engine):
    """Every optimizer step (any torch.optim optimizer) marks the foreign-optimizer engines' compute
    copies stale; the next forward refreshes them."""
    global _FOREIGN_ENGINES
    import weakref
    if _FOREIGN_ENGINES is None:
        _FOREIGN_ENGINES = weakref.WeakSet()

        def after_step(_opt, _args, _kwargs):
            for e in list(_FOREIGN_ENGINES):
                e._params_dirty = True
        from torch.optim.optimizer import register_optimizer_step_post_hook
        register_optimizer_step_post_hook(after_step)
    _FOREIGN_ENGINES.add(engine)


class _GradBucket:
    """torch.distributed.GradBucket's interface over one bucket of the flat gradient buffer."""

    def __init__(self, engine: DataParallel, b: int):
        self._e, self._b = engine, b
        lo, hi = engine.bucket_ranges[b]
        self._buf = engine.flat.grad[lo:hi]

    def index(self) -> int:
        return self._b

    def buffer(self) -> torch.Tensor:
        return self._buf

    def set_buffer(self, t: torch.Tensor):
        self._buf.copy_(t.reshape(-1))

    def is_last(self) -> bool:
        return self._b == len(self._e.buckets) - 1

    def parameters(self):
        return [self._e.flat.params[i] for i in self._e.buckets[self._b]]

    def gradients(self):
        return [p.grad for p in self.parameters()]


class FlatSGD:
    """torch.optim.SGD semantics over the flat buffer in ONE fused kernel launch
    (momentum + weight decay + 1/world + bf16 copy refresh)."""

    def __init__(self, engine: DataParallel, lr: float, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False):
        self.engine = engine
        self.lr, self.momentum, self.dampening = lr, momentum, dampening
        self.weight_decay, self.nesterov = weight_decay, nesterov
        # shard mode: momentum only for this rank's shards, packed (1/world of the optimizer state)
        self.segments = []  # (flat lo, flat hi, momentum offset)
        off = 0
        for lo, hi in engine.shard_ranges if engine.sharded else [(0, engine.flat.numel)]:
            self.segments.append((lo, hi, off))
            off += hi - lo
        self.momentum_buf = torch.zeros(off, dtype=torch.float32, device=engine.flat.data.device) if momentum else None
        self.steps = 0
        self.param_groups = [dict(lr=lr, momentum=momentum, weight_decay=weight_decay, nesterov=nesterov,
                                  dampening=dampening)]

    def zero_grad(self, set_to_none: bool = False):
        self.engine.zero_grad()

    def step(self):
        from mi355x_dp.ops.functional import sgd_flat_
        self.engine.finish_gradient_sync(average=False)
        g = self.param_groups[0]
        f = self.engine.flat
        for lo, hi, mo in self.segments:
            mom = self.momentum_buf[mo:mo + hi - lo] if self.momentum_buf is not None else None
            sgd_flat_(f.data[lo:hi], f.grad[lo:hi], mom, f.bf16[lo:hi] if f.bf16 is not None else None, g["lr"],
                      g["momentum"], g["dampening"], g["weight_decay"], g["nesterov"], first_step=(self.steps == 0),
                      grad_scale=self.engine.grad_scale)
        if self.engine.sharded and self.engine.comm_on:
            self.engine.gather_params()  # bf16 copy + transposed operands refreshed after the gather
        else:
            f.refresh_transposed()  # dgrad operands of every conv, one launch
        self.steps += 1

    def state_dict(self):
        """In shard mode ``momentum_buf`` is this rank's packed shards (a per-rank optimizer
        checkpoint, tagged with ``shard``)."""
        sd = {"steps": self.steps, "param_groups": self.param_groups,
              "momentum_buf": self.momentum_buf.detach().cpu() if self.momentum_buf is not None else None}
        if self.engine.sharded:
            sd["shard"] = self._shard_meta()
        return sd

    def _shard_meta(self):
        """Which slice of the packed momentum belongs to which flat range: the bucket plan (flat
        [lo, hi) of every bucket and of this rank's shard of it) depends on the planner settings
        and, with calibrate=True, on timing -- a resume must see the same plan."""
        e = self.engine
        return {"rank": e.rank, "world": e.world_size, "numel": int(e.flat.numel),
                "bucket_ranges": [[int(lo), int(hi)] for lo, hi in e.bucket_ranges],
                "shard_ranges": [[int(lo), int(hi)] for lo, hi in e.shard_ranges]}

    def load_state_dict(self, sd):
        if self.engine.sharded:
            want, got = self._shard_meta(), sd.get("shard") or {}
            if {k: got.get(k) for k in ("rank", "world")} != {"rank": want["rank"], "world": want["world"]}:
                raise ValueError(f"optimizer shard (rank {got.get('rank')} of {got.get('world')}) does not match "
                                 f"this rank ({want['rank']} of {want['world']})")
            for k in ("numel", "bucket_ranges", "shard_ranges"):
                if got.get(k) != want[k]:
                    raise ValueError(f"optimizer shard checkpoint was written with a different bucket plan ({k} "
                                     "differs): its packed momentum would pair with the wrong parameters; resume "
                                     "with the same bucket_cap_mb / first / last / min bucket settings and without "
                                     "calibrate=True")
        self.steps = sd["steps"]
        self.param_groups = sd["param_groups"]
        if sd.get("momentum_buf") is not None and self.momentum_buf is not None:
            self.momentum_buf.copy_(sd["momentum_buf"])
