"""Flat parameter / gradient storage.

All trainable parameters of a model are re-homed into ONE contiguous fp32
master buffer (plus matching fp32 gradient buffer and a bf16 compute copy),
laid out in reverse registration order (= approximate backward order), each
tensor aligned to 64 elements.  4-D conv weights are stored ``[K][R][S][C]``
(the ``channels_last`` strides of a ``[K, C, R, S]`` tensor) which is the
layout the MFMA conv kernels consume, so the bf16 copy refreshed by the fused
SGD kernel is directly the kernel operand.  Parameter objects are kept (their
``.data`` is re-pointed), so optimizers/state_dict/named_parameters behave as
before; ``state_dict`` hooks write NCHW-contiguous tensors.

This replaces the reference's per-tensor DDP bucket copy-in/copy-out
(SURVEY.md §2.5 K14, §3.2): buckets are slices of the gradient buffer, the
backward kernels accumulate straight into them, and the all-reduce runs on
the slice in place.
"""
from __future__ import annotations

from typing import List, Sequence

import torch

ALIGN = 64  # elements (256 B for fp32)


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def _kernel_view(flat: torch.Tensor, off: int, shape, kernel_layout: bool = True) -> torch.Tensor:
    n = 1
    for s in shape:
        n *= s
    v = flat[off:off + n]
    if len(shape) == 4 and kernel_layout:
        K, C, R, S = shape
        return v.view(K, R, S, C).permute(0, 3, 1, 2)
    return v.view(shape)


class FlatParams:
    """Owns the flat fp32 params, fp32 grads and bf16 copy for a list of parameters."""

    def __init__(self, params: Sequence[torch.nn.Parameter], bf16_copy: bool = True, kernel_layout_ids=None,
                 group_ends=(), group_align: int = ALIGN):
        """``kernel_layout_ids``: ids of 4-D params consumed by the native conv kernels; they are
        stored [K][R][S][C].  Every other parameter keeps PyTorch's default contiguous layout (a
        stock nn.Conv2d would otherwise start producing channels_last outputs).  ``None`` = all.
        ``group_ends``: indices of parameters that close a gradient bucket; the offset after each
        is rounded up to ``group_align`` elements (balanced-shard mode: every bucket a multiple of
        world x 64 elements, so its reduce-scatter shards are equal and aligned)."""
        params = [p for p in params if p.requires_grad]
        if not params:
            raise ValueError("no trainable parameters")
        dev = params[0].device
        self.device = dev
        self.params: List[torch.nn.Parameter] = list(params)
        self.kernel_layout = [kernel_layout_ids is None or id(p) in kernel_layout_ids for p in self.params]
        self.offsets = []
        off = 0
        ends = set(group_ends)
        for i, p in enumerate(self.params):
            self.offsets.append(off)
            off += _align(p.numel())
            if i in ends:
                off = (off + group_align - 1) // group_align * group_align
        self.numel = off
        self.data = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.bf16 = torch.zeros(off, dtype=torch.bfloat16, device=dev) if bf16_copy else None
        with torch.no_grad():
            for p, o, kl in zip(self.params, self.offsets, self.kernel_layout):
                v = _kernel_view(self.data, o, tuple(p.shape), kl)
                v.copy_(p.data)
                p.data = v
                p.grad = _kernel_view(self.grad, o, tuple(p.shape), kl)
                p._mi_flat = True
                if self.bf16 is not None:
                    p._mi_bf16 = _kernel_view(self.bf16, o, tuple(p.shape), kl)
            if self.bf16 is not None:
                from mi355x_dp.ops.functional import cast_bf16_
                cast_bf16_(self.data, self.bf16)
        self._init_transposed()

    def _init_transposed(self):
        """Data-gradient operands: every kernel-layout conv weight [K][R][S][C] also kept transposed
        as [C][R][S][K], and every Linear weight [N][K] as [K][N], in a second bf16 buffer (same
        offsets), rebuilt for ALL of them by ONE kernel launch whenever the bf16 copy changes
        (``refresh_transposed``), instead of one transpose per layer per backward.  Attached as
        ``p._mi_bf16_t``; GPU + native kernels only."""
        self.bf16_t = None
        if self.bf16 is None or self.device.type != "cuda":
            return
        from mi355x_dp.ops import _lib
        if _lib.load(required=False) is None:
            return
        desc, blk = [], 0
        for p, o, kl in zip(self.params, self.offsets, self.kernel_layout):
            if self._transposed(p, kl):
                K, C, R, S = p.shape if p.dim() == 4 else (p.shape[0], p.shape[1], 1, 1)
                desc.append([o, o, K, R * S, C, blk])
                blk += R * S * ((K + 63) // 64) * ((C + 63) // 64)
        if not desc:
            return
        self.bf16_t = torch.zeros_like(self.bf16)
        self._wt_desc = torch.tensor(desc, dtype=torch.int32, device=self.device)
        self._wt_blocks = blk
        for p, o, kl in zip(self.params, self.offsets, self.kernel_layout):
            if self._transposed(p, kl):
                if p.dim() == 4:
                    K, C, R, S = p.shape
                    p._mi_bf16_t = self.bf16_t[o:o + p.numel()].view(C, R, S, K)
                else:  # Linear weight [out][in] -> W^T [in][out], the data-gradient GEMM operand
                    p._mi_bf16_t = self.bf16_t[o:o + p.numel()].view(p.shape[1], p.shape[0])
        self.refresh_transposed()

    @staticmethod
    def _transposed(p, kernel_layout) -> bool:
        """kernel-layout conv weights and Linear weights (both dims multiples of 8) get a cached
        transposed bf16 copy."""
        if p.dim() == 4:
            return kernel_layout
        return p.dim() == 2 and p.shape[0] % 8 == 0 and p.shape[1] % 8 == 0

    def refresh_transposed(self):
        if getattr(self, "bf16_t", None) is None:
            return
        from mi355x_dp.ops._lib import call, ptr, stream_of
        call("mi_conv_wtrans_multi", ptr(self.bf16), ptr(self.bf16_t), ptr(self._wt_desc), len(self._wt_desc),
             self._wt_blocks, stream_of(self.bf16))

    def param_range(self, i: int):
        p = self.params[i]
        return self.offsets[i], self.offsets[i] + p.numel()

    def zero_grad(self):
        self.grad.zero_()

    def refresh_bf16(self):
        if self.bf16 is not None:
            from mi355x_dp.ops.functional import cast_bf16_
            cast_bf16_(self.data, self.bf16)
            self.refresh_transposed()

    def reattach_grads(self) -> bool:
        """Re-point .grad at the flat views (after user code set them to None, e.g. a stock
        optimizer's ``zero_grad(set_to_none=True)``).  Returns True if any was re-pointed."""
        views = getattr(self, "_grad_views", None)
        if views is None:
            views = self._grad_views = [_kernel_view(self.grad, o, tuple(p.shape), kl)
                                        for p, o, kl in zip(self.params, self.offsets, self.kernel_layout)]
        changed = False
        for p, v in zip(self.params, views):
            g = p.grad
            if g is None or g.data_ptr() != v.data_ptr():
                p.grad = v
                changed = True
        return changed

    def params_version(self) -> int:
        """Sum of the parameters' autograd version counters: changes whenever anything (a stock
        optimizer's step, an in-place update) writes a parameter in place."""
        return sum(p._version for p in self.params)


class FlatBuffers:
    """Flat fp32 storage for floating-point module buffers (BN running stats) so the
    per-forward ``broadcast_buffers`` of DDP is one collective."""

    def __init__(self, buffers: Sequence[torch.Tensor]):
        self.buffers = [b for b in buffers if b.is_floating_point()]
        self.others = [b for b in buffers if not b.is_floating_point()]
        n = sum(b.numel() for b in self.buffers)
        dev = self.buffers[0].device if self.buffers else torch.device("cpu")
        self.data = torch.zeros(max(n, 1), dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for b in self.buffers:
                v = self.data[off:off + b.numel()].view(b.shape)
                v.copy_(b)
                b.data = v
                off += b.numel()
