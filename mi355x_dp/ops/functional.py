"""Autograd functions over the native gfx950 kernels.

Device contract (GPU path): activations are bf16 tensors in ``channels_last``
memory format (NHWC storage), conv weights are read as bf16 ``[K][R][S][C]``
(= channels_last storage of a ``[K, C, R, S]`` tensor), accumulation is fp32.
Host tensors take the fp32 PyTorch reference path (used by the CPU tests and
the gloo CPU configuration) -- the two paths are selected by device, never by
availability: a CUDA tensor without the native library is an error.

Gradient sinks: a parameter registered with a flat-buffer engine
(``mi355x_dp.parallel.flat``) carries ``_mi_flat = True``; its ``.grad`` is a
view into the engine's fp32 gradient buffer and our backward kernels
accumulate straight into it (split-K atomics / ``+=``), then signal the engine
via ``_mi_on_grad_ready`` so the bucket all-reduce can start while backward
continues.  Any other parameter gets a freshly allocated gradient returned
through autograd as usual (works with stock ``torch.nn.parallel.DDP``).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.nn.functional as F

from . import _lib
from . import kernels as _k  # noqa: F401  (registers signatures)
from ._lib import ptr, stream_of

CL = torch.channels_last
BF16 = torch.bfloat16


# --------------------------------------------------------------------- helpers
def _nhwc(x: torch.Tensor) -> torch.Tensor:
    if x.dtype != BF16:
        x = x.to(BF16)
    if x.dim() == 4 and not x.is_contiguous(memory_format=CL):
        x = x.contiguous(memory_format=CL)
    return x


def weight_bf16(w: torch.Tensor) -> torch.Tensor:
    """bf16 compute copy of a parameter in kernel layout (flat-engine shadow if present)."""
    w16 = getattr(w, "_mi_bf16", None)
    if w16 is not None:
        return w16
    with torch.no_grad():
        if w.dim() == 4:
            return w.detach().to(BF16).contiguous(memory_format=CL)
        return w.detach().to(BF16).contiguous()


def weight_bf16_t(w: torch.Tensor) -> torch.Tensor:
    """Conv-dgrad operand [C][R][S][K] (bf16) of a [K, C, R, S] conv weight: the flat engine's
    transposed copy (refreshed once per optimizer step for every conv) or a fresh transpose."""
    wt = getattr(w, "_mi_bf16_t", None)
    if wt is not None:
        return wt
    K, C, R, S = w.shape
    w16 = weight_bf16(w)
    wt = torch.empty((C, R, S, K), dtype=BF16, device=w.device)
    _lib.call("mi_conv_wtrans", ptr(w16), ptr(wt), K, R * S, C, stream_of(w16))
    return wt


def linear_weight_t(w: torch.Tensor) -> torch.Tensor:
    """Linear data-gradient operand W^T [in][out] (bf16): the flat engine's cached transpose
    (refreshed once per optimizer step) or a fresh one."""
    wt = getattr(w, "_mi_bf16_t", None)
    if wt is not None and wt.dim() == 2:
        return wt
    return weight_bf16(w).t().contiguous()


def _flat(p) -> bool:
    return p is not None and getattr(p, "_mi_flat", False) and p.grad is not None


def _grad_buffer(p: torch.Tensor) -> torch.Tensor:
    """fp32 gradient target in kernel layout: the engine's view, or a fresh zero tensor."""
    if _flat(p):
        return p.grad
    if p.dim() == 4:
        return torch.zeros_like(p, dtype=torch.float32, memory_format=CL)
    return torch.zeros_like(p, dtype=torch.float32)


class WgradStream:
    """Weight gradients on a side HIP stream (owned by the flat-buffer engine, one per device).

    A conv's weight gradient is needed by nothing but the optimizer, while its data gradient is
    the critical path of backward; on one stream every kernel's tail (its last, partly filled
    wave of workgroups) and every small split-K reduce / BN finalize idles most of the 256 CUs.
    With the weight gradients on their own stream the two chains overlap and fill each other's
    tails.  Ordering rules (no host synchronisation anywhere):

    * ``run``: the side stream waits for the compute stream (the kernel's operands were produced
      there), the weight-gradient kernels run on it, their operands are ``record_stream``-ed so
      the caching allocator does not recycle them early, and the parameter is marked ready ON
      the side stream -- so a bucket's collective (which waits on the current stream) waits for
      the side stream, which itself has waited for everything the compute stream did before;
    * marks of gradients produced on the compute stream (BN affine) while side work is pending
      are deferred and issued on the side stream at its next ``run`` (or ``join``), for the same
      reason: a bucket may mix both kinds;
    * ``join`` (engine: before the optimizer / reducer finish, at forward, at zero_grad) makes
      the compute stream wait for the side stream.
    Disabled inside HIP graph capture (the captured step stays single-stream)."""

    _streams = {}  # device index -> the side stream (shared by every engine on that device)

    def __init__(self, device):
        self.device = torch.device(device)
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        if idx not in WgradStream._streams:
            # MI355X_DP_WGRAD_PRIORITY=-1: the side stream's workgroups are dispatched ahead of the
            # compute stream's (default 0: equal priority; profiles/rn50_bs256_wgrad_stream.md)
            with torch.cuda.device(idx):
                cus = int(os.environ.get("MI355X_DP_WGRAD_CUS", "0"))
                if cus > 0:
                    # A/B knob: the side stream confined to `cus` CUs (spread over the CU ids; the
                    # compute stream keeps every CU), MI355X_DP_WGRAD_CU_BLOCK=1: the first `cus` ids
                    h = ctypes.c_void_p()
                    _lib.call("mi_create_cu_masked_stream", cus, int(os.environ.get("MI355X_DP_WGRAD_CU_BLOCK", "0")
                                                                      != "1"), ctypes.addressof(h))
                    st = torch.cuda.ExternalStream(h.value, device=self.device)
                else:
                    st = torch.cuda.Stream(device=self.device,
                                           priority=int(os.environ.get("MI355X_DP_WGRAD_PRIORITY", "0")))
                # its own split-K slab workspace (gemm_conv.hip)
                _lib.call("mi_register_wgrad_stream", ctypes.c_void_p(st.cuda_stream))
            WgradStream._streams[idx] = st
        self.stream = WgradStream._streams[idx]
        self.dirty = False
        self.deferred = []
        self.runs = 0

    # > 0 while a GraphedStep warms up / captures: the captured step is single-stream, and its
    # warm-up must run the same kernels on the same stream so the native library's lazily sized
    # workspaces exist before capture (no allocation may happen inside it)
    suspended = 0

    def active(self) -> bool:
        return WgradStream.suspended == 0 and not torch.cuda.is_current_stream_capturing()

    def run(self, fn, tensors=(), cb=None):
        main = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(main)
        with torch.cuda.stream(self.stream):
            out = fn()
            for t in tensors:
                if t is not None:
                    t.record_stream(self.stream)
            self.dirty = True
            self.runs += 1
            self._flush_locked()
            if cb is not None:
                cb()
        return out

    def _flush_locked(self):
        pending, self.deferred = self.deferred, []
        for d in pending:
            d()

    def mark(self, cb):
        if self.dirty:
            self.deferred.append(cb)
        else:
            cb()

    def join(self):
        if self.deferred:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                self._flush_locked()
        if self.dirty:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            self.dirty = False


def _side(p):
    """the engine's weight-gradient stream for parameter p, if it should be used now"""
    s = getattr(p, "_mi_side", None)
    if s is None or not _flat(p) or not s.active():
        return None
    return s


def _finish_grad(p: torch.Tensor, g: torch.Tensor):
    """Return value for autograd: None if accumulated in place (flat engine)."""
    if _flat(p):
        cb = getattr(p, "_mi_on_grad_ready", None)
        if cb is not None:
            s = getattr(p, "_mi_side", None)
            if s is not None:
                s.mark(cb)
            else:
                cb()
        return None
    return g.to(p.dtype) if g.dtype != p.dtype else g


def run_wgrad(p: torch.Tensor, fn, tensors=()):
    """Run ``fn`` (which writes p's fp32 gradient into the flat buffer) on the engine's weight-
    gradient stream when there is one, else inline; then signal the engine (see WgradStream)."""
    s = _side(p)
    if s is None:
        fn()
        return
    s.run(fn, tensors, getattr(p, "_mi_on_grad_ready", None))


def _conv_out(h, r, stride, pad):
    return (h + 2 * pad - r) // stride + 1


# ======================================================================= conv
def pad_channels8(x: torch.Tensor) -> torch.Tensor:
    """[N, C<=8, H, W] -> bf16 channels_last [N, 8, H, W] (zero channels appended): one 16-byte
    chunk per pixel, the layout the small-channel (stem) conv mode of the MFMA kernel gathers."""
    N, C, H, W = x.shape
    out = torch.empty((N, 8, H, W), dtype=BF16, device=x.device, memory_format=CL)
    out[:, C:].zero_()
    out[:, :C].copy_(x)
    return out


class _Conv2d(torch.autograd.Function):
    """Implicit-GEMM convolution.  Paths (chosen by channel count, all MFMA):
      direct : C % 64 == 0                      (every ResNet conv but the stem)
      c8     : C <= 8, input padded to 8 channels (the 7x7 stem: one 16-B chunk = one tap)
      col    : other C (explicit im2col + GEMM)"""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, stats):
        N, C, H, W = x.shape
        K, Cw, R, S = weight.shape
        P, Q = _conv_out(H, R, stride, padding), _conv_out(W, S, stride, padding)
        w16 = weight_bf16(weight)
        if C <= 8 and C % 64 != 0:
            if C != 8:
                x = pad_channels8(x)
                C = 8
            mode = "c8"
        elif C % 64 == 0:
            mode = "direct"
        else:
            mode = "col"
        x = _nhwc(x)
        st = stream_of(x)
        y = torch.empty((N, K, P, Q), dtype=BF16, device=x.device, memory_format=CL)
        saved = x
        if mode == "direct":
            _lib.call("mi_conv2d_fwd", ptr(x), ptr(w16), ptr(y), ptr(None), ptr(stats), N, H, W, C, K, R, S,
                      stride, padding, P, Q, 0, st)
        elif mode == "c8":
            wp = torch.zeros((K, R, S, 8), dtype=BF16, device=x.device)
            wp[..., :Cw].copy_(w16.permute(0, 2, 3, 1))
            _lib.call("mi_conv2d_fwd", ptr(x), ptr(wp), ptr(y), ptr(None), ptr(stats), N, H, W, 8, K, R, S,
                      stride, padding, P, Q, 0, st)
        else:
            # explicit im2col (k = (r*S+s)*C + c) + MFMA GEMM
            Kr = R * S * C
            Kp = (Kr + 7) // 8 * 8
            col = torch.empty((N * P * Q, Kp), dtype=BF16, device=x.device)
            _lib.call("mi_im2col", ptr(x), ptr(col), N, H, W, C, R, S, stride, padding, P, Q, Kp, st)
            wp = torch.zeros((K, Kp), dtype=BF16, device=x.device)
            wp[:, :Kr].copy_(w16.permute(0, 2, 3, 1).reshape(K, Kr))
            _lib.call("mi_gemm_nt", ptr(col), ptr(wp), ptr(y), ptr(None), ptr(stats), N * P * Q, K, Kp, Kp, Kp, K,
                      0, 0, st)
            saved = col
        if bias is not None:
            y = y + bias.to(BF16).view(1, K, 1, 1)
        ctx.geom = (N, C, H, W, K, Cw, R, S, stride, padding, P, Q)
        ctx.has_bias = bias is not None
        ctx.bias_param = bias
        ctx.mode = mode
        ctx.save_for_backward(saved, weight, w16)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W, K, Cw, R, S, stride, padding, P, Q = ctx.geom
        xs, weight, w16 = ctx.saved_tensors
        dy = _nhwc(dy)
        st = stream_of(dy)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if ctx.mode != "direct":
                raise NotImplementedError("input gradient of a small-channel (stem) convolution")
            wt = weight_bf16_t(weight)
            dx = torch.empty((N, C, H, W), dtype=BF16, device=dy.device, memory_format=CL)
            _lib.call("mi_conv2d_dgrad", ptr(dy), ptr(wt), ptr(dx), N, H, W, C, K, R, S, stride, padding, P, Q, st)
        if ctx.needs_input_grad[1]:
            g = _grad_buffer(weight)
            on_side = ctx.mode == "direct" and _side(weight) is not None
            if on_side:
                # flat engine with a weight-gradient stream: kernels + ready signal on the side stream
                run_wgrad(weight, lambda: _lib.call("mi_conv2d_wgrad", ptr(xs), ptr(dy), ptr(g), N, H, W, C, K, R,
                                                    S, stride, padding, P, Q, stream_of(dy)), (xs, dy))
            elif ctx.mode == "direct":
                _lib.call("mi_conv2d_wgrad", ptr(xs), ptr(dy), ptr(g), N, H, W, C, K, R, S, stride, padding, P, Q, st)
            elif ctx.mode == "c8":
                gp = torch.zeros((K, R, S, 8), dtype=torch.float32, device=dy.device)
                _lib.call("mi_conv2d_wgrad", ptr(xs), ptr(dy), ptr(gp), N, H, W, 8, K, R, S, stride, padding, P, Q,
                          st)
                g.add_(gp[..., :Cw].permute(0, 3, 1, 2))
            else:
                Kr = R * S * C
                Kp = xs.shape[1]
                gp = torch.zeros((K, Kp), dtype=torch.float32, device=dy.device)
                _lib.call("mi_gemm_tn", ptr(dy), ptr(xs), ptr(gp), K, Kp, N * P * Q, K, Kp, Kp, st)
                g.add_(gp[:, :Kr].reshape(K, R, S, C).permute(0, 3, 1, 2))
            if not on_side:
                dw = _finish_grad(weight, g)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            bias = ctx.bias_param
            gb = _grad_buffer(bias)
            if K % 8 == 0:  # dy is NHWC storage: a [N*P*Q][K] row-major matrix
                _lib.call("mi_colsum_bf16", ptr(dy), ptr(gb), N * P * Q, K, K, st)
            else:
                gb.add_(dy.float().sum(dim=(0, 2, 3)))
            db = _finish_grad(bias, gb)
        return dx, dw, db, None, None, None


def conv2d(x, weight, bias=None, stride=1, padding=0):
    if not x.is_cuda:
        return F.conv2d(x, weight, bias, stride, padding)
    return _Conv2d.apply(x, weight, bias, stride, padding, None)


def conv2d_with_stats(x, weight, stride=1, padding=0):
    """Conv (no bias) whose epilogue also writes per-channel (sum, sumsq) partials of its bf16
    output -> (y, (slab, rows)); feeds ``batch_norm_act(..., stats=...)`` so BN skips its own
    statistics pass over y (one full read of the activation saved per BN layer)."""
    N, C, H, W = x.shape
    K, _, R, S = weight.shape
    P, Q = _conv_out(H, R, stride, padding), _conv_out(W, S, stride, padding)
    lib = _lib.load()
    rows = lib.mi_conv_stat_rows_g(N, H, W, C if C % 64 == 0 else 8, K, R, S, stride, padding, P, Q)
    slab = torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, K), dtype=torch.float32, device=x.device)
    y = _Conv2d.apply(x, weight, None, stride, padding, slab)
    return y, (slab, rows)


# ================================================================ batch norm
class _BatchNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, nbt, training, momentum, eps, relu,
                stats):
        N, C, H, W = x.shape
        M = N * H * W
        x = _nhwc(x)
        res = _nhwc(residual) if residual is not None else None
        st = stream_of(x)
        dev = x.device
        y = torch.empty_like(x, memory_format=CL)
        f32 = dict(dtype=torch.float32, device=dev)
        scale = torch.empty(C, **f32)
        shift = torch.empty(C, **f32)
        if training:
            if stats is not None:
                part, pre_rows = stats
            else:
                lib = _lib.load()
                part = torch.empty((lib.mi_bn_partial_rows(M, C) + lib.mi_bn_slab_extra_rows(), 2, C), **f32)
                pre_rows = 0
            mean = torch.empty(C, **f32)
            invstd = torch.empty(C, **f32)
            _lib.call("mi_bn_fwd_train", ptr(x), ptr(res), ptr(y), M, C, float(eps), float(momentum),
                      ptr(weight), ptr(bias), ptr(running_mean), ptr(running_var), ptr(nbt), ptr(mean),
                      ptr(invstd), ptr(scale), ptr(shift), ptr(part), int(pre_rows), int(relu), st)
        else:
            mean = invstd = None
            _lib.call("mi_bn_fwd_eval", ptr(x), ptr(res), ptr(y), M, C, float(eps), ptr(weight), ptr(bias),
                      ptr(running_mean), ptr(running_var), ptr(scale), ptr(shift), int(relu), st)
        ctx.training = training
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, y, weight, bias, mean, invstd, scale)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, weight, bias, mean, invstd, scale = ctx.saved_tensors
        dy = _nhwc(dy)
        N, C, H, W = x.shape
        M = N * H * W
        st = stream_of(dy)
        dev = dy.device
        dx = torch.empty_like(x, memory_format=CL)
        dres = torch.empty_like(x, memory_format=CL) if (ctx.has_res and ctx.needs_input_grad[3]) else None
        dw = db = None
        if ctx.training:
            gw = _grad_buffer(weight) if (weight is not None and ctx.needs_input_grad[1]) else None
            gb = _grad_buffer(bias) if (bias is not None and ctx.needs_input_grad[2]) else None
            lib = _lib.load()
            nblk = lib.mi_bn_partial_rows(M, C) + lib.mi_bn_slab_extra_rows()
            part = torch.empty((nblk, 2, C), dtype=torch.float32, device=dev)
            coef = torch.empty((3, C), dtype=torch.float32, device=dev)
            _lib.call("mi_bn_bwd_train", ptr(dy), ptr(y), ptr(x), ptr(dx), ptr(dres), M, C, ptr(weight), ptr(mean),
                      ptr(invstd), ptr(gw), ptr(gb), ptr(coef), ptr(part), int(ctx.relu), st)
            if gw is not None:
                dw = _finish_grad(weight, gw)
            if gb is not None:
                db = _finish_grad(bias, gb)
        else:
            _lib.call("mi_bn_bwd_eval", ptr(dy), ptr(y), ptr(scale), ptr(dx), ptr(dres), M, C, int(ctx.relu), st)
        return dx, dw, db, dres, None, None, None, None, None, None, None, None


def batch_norm_act(x, weight, bias, running_mean, running_var, num_batches_tracked, training, momentum, eps,
                   relu=False, residual=None, stats=None):
    """y = act(BN(x) + residual).  ``momentum=None`` (cumulative average) is resolved by the caller."""
    if not x.is_cuda:
        y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
        if training and num_batches_tracked is not None:
            num_batches_tracked.add_(1)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y
    if not training and running_mean is None:
        raise ValueError("eval-mode batch_norm without running statistics")
    return _BatchNormAct.apply(x, weight, bias, residual, running_mean, running_var,
                               num_batches_tracked if training else None, bool(training), float(momentum),
                               float(eps), bool(relu), stats if training else None)


# ==================================================================== pooling
class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        N, C, H, W = x.shape
        P, Q = _conv_out(H, k, s, pad), _conv_out(W, k, s, pad)
        x = _nhwc(x)
        y = torch.empty((N, C, P, Q), dtype=BF16, device=x.device, memory_format=CL)
        idx = torch.empty((N, P, Q, C), dtype=torch.uint8, device=x.device)
        _lib.call("mi_maxpool_fwd", ptr(x), ptr(y), ptr(idx), N, H, W, C, P, Q, k, s, pad, stream_of(x))
        ctx.save_for_backward(idx)
        ctx.geom = (N, C, H, W, P, Q, k, s, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W, P, Q, k, s, pad = ctx.geom
        dy = _nhwc(dy)
        dx = torch.empty((N, C, H, W), dtype=BF16, device=dy.device, memory_format=CL)
        _lib.call("mi_maxpool_bwd", ptr(dy), ptr(idx), ptr(dx), N, H, W, C, P, Q, k, s, pad, stream_of(dy))
        return dx, None, None, None


def max_pool2d(x, kernel_size=3, stride=2, padding=1):
    if not x.is_cuda:
        return F.max_pool2d(x, kernel_size, stride, padding)
    return _MaxPool.apply(x, int(kernel_size), int(stride), int(padding))


class _GlobalAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        x = _nhwc(x)
        y = torch.empty((N, C), dtype=BF16, device=x.device)
        _lib.call("mi_gap_fwd", ptr(x), ptr(y), N, H * W, C, stream_of(x))
        ctx.geom = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.geom
        dy = dy.to(BF16).contiguous()
        dx = torch.empty((N, C, H, W), dtype=BF16, device=dy.device, memory_format=CL)
        _lib.call("mi_gap_bwd", ptr(dy), ptr(dx), N, H * W, C, stream_of(dy))
        return dx


def global_avg_pool(x):
    """[N,C,H,W] -> [N,C]  (AdaptiveAvgPool2d(1) + flatten)."""
    if not x.is_cuda:
        return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
    return _GlobalAvgPool.apply(x)


# ===================================================================== linear
class _Linear(torch.autograd.Function):
    """y = x W^T + b on MFMA GEMMs; output fp32.  Feature dims that are not a multiple
    of 8 (e.g. a 10-class head) are zero-padded to the 16-byte vector granule."""

    @staticmethod
    def forward(ctx, x, weight, bias, out_bf16=False):
        x2 = x.reshape(-1, x.shape[-1])
        if x2.dtype != BF16:
            x2 = x2.to(BF16)
        x2 = x2.contiguous()
        M, Kd = x2.shape
        N = weight.shape[0]
        if Kd % 8:
            raise NotImplementedError("native linear needs in_features % 8 == 0")
        Np = (N + 7) // 8 * 8
        w16 = weight_bf16(weight)
        bp = bias
        if Np != N:
            wp = torch.zeros((Np, Kd), dtype=BF16, device=x.device)
            wp[:N].copy_(w16)
            w16 = wp
            if bias is not None:
                bp = torch.zeros(Np, dtype=torch.float32, device=x.device)
                bp[:N].copy_(bias)
        y = torch.empty((M, Np), dtype=BF16 if out_bf16 else torch.float32, device=x.device)
        _lib.call("mi_gemm_nt", ptr(x2), ptr(w16), ptr(y), ptr(bp), ptr(None), M, Np, Kd, Kd, Kd, Np,
                  0 if out_bf16 else 1, 0, stream_of(x))
        if Np != N:
            y = y[:, :N].contiguous()
        ctx.save_for_backward(x2, weight, w16)
        ctx.bias_param = bias
        ctx.has_bias = bias is not None
        ctx.in_shape = x.shape
        ctx.in_dtype = x.dtype
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, w16 = ctx.saved_tensors  # w16 is [Np][Kd] (padded if needed)
        M, Kd = x2.shape
        N = weight.shape[0]
        Np = w16.shape[0]
        dy2 = dy.reshape(M, N)
        gb32 = None
        if Np != N:
            dyp = torch.zeros((M, Np), dtype=BF16, device=dy.device)
            dyp[:, :N].copy_(dy2)
            dy2 = dyp
        elif dy2.dtype == torch.float32 and dy2.is_contiguous() and N % 8 == 0:
            # fp32 logits gradient: one native pass casts it to the bf16 GEMM operand and sums the
            # bias gradient from the fp32 values
            d16 = torch.empty((M, N), dtype=BF16, device=dy.device)
            if ctx.has_bias and ctx.needs_input_grad[2]:
                gb32 = _grad_buffer(ctx.bias_param)
            _lib.call("mi_cast_colsum_f32", ptr(dy2), ptr(d16), ptr(gb32), M, N, stream_of(dy))
            dy2 = d16
        else:
            dy2 = dy2.to(BF16).contiguous()
        st = stream_of(dy)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            # dX[M][Kd] = dY[M][Np] * W[Np][Kd]  ->  NT with B = W^T [Kd][Np]
            wt = linear_weight_t(weight) if Np == N else w16.t().contiguous()
            dxf = torch.empty((M, Kd), dtype=BF16, device=dy.device)
            _lib.call("mi_gemm_nt", ptr(dy2), ptr(wt), ptr(dxf), ptr(None), ptr(None), M, Kd, Np, Np, Np, Kd, 0, 0, st)
            dx = dxf.reshape(ctx.in_shape).to(ctx.in_dtype)
        if ctx.needs_input_grad[1]:
            g = _grad_buffer(weight)
            if Np == N:
                _lib.call("mi_gemm_tn", ptr(dy2), ptr(x2), ptr(g), N, Kd, M, N, Kd, Kd, st)
            else:
                gp = torch.zeros((Np, Kd), dtype=torch.float32, device=dy.device)
                _lib.call("mi_gemm_tn", ptr(dy2), ptr(x2), ptr(gp), Np, Kd, M, Np, Kd, Kd, st)
                g.add_(gp[:N])
            dw = _finish_grad(weight, g)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            bias = ctx.bias_param
            gb = gb32 if gb32 is not None else _grad_buffer(bias)  # gb32: summed by the cast pass
            if gb32 is None and dy2.dtype == BF16 and Np == N and dy.dtype == BF16:
                _lib.call("mi_colsum_bf16", ptr(dy2), ptr(gb), M, N, N, st)
            elif gb32 is None:
                gb.add_(dy.reshape(M, N).float().sum(0))
            db = _finish_grad(bias, gb)
        return dx, dw, db, None


def linear(x, weight, bias=None, out_bf16=False):
    """MFMA GEMM linear layer; ``out_bf16`` keeps activations bf16 (transformer internals),
    otherwise fp32 output (classifier heads / logits)."""
    if not x.is_cuda:
        return F.linear(x, weight, bias)
    return _Linear.apply(x, weight, bias, bool(out_bf16))


# ============================================================= cross entropy
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target):
        lg = logits.float().contiguous()
        N, ncls = lg.shape
        tgt = target.to(torch.int64).contiguous()
        lse = torch.empty(2 * N, dtype=torch.float32, device=lg.device)  # [lse rows | per-row losses]
        loss = torch.empty((), dtype=torch.float32, device=lg.device)
        _lib.call("mi_ce_fwd", ptr(lg), ptr(tgt), ptr(lse), ptr(loss), N, ncls, ncls, stream_of(lg))
        ctx.save_for_backward(lg, tgt, lse)
        ctx.in_dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, gout):
        lg, tgt, lse = ctx.saved_tensors
        N, ncls = lg.shape
        g = gout.float().contiguous().reshape(1)
        f32 = ctx.in_dtype == torch.float32  # the gradient in the logits' dtype: no autograd cast launch
        dl = torch.empty((N, ncls), dtype=torch.float32 if f32 else BF16, device=lg.device)
        _lib.call("mi_ce_bwd", ptr(lg), ptr(tgt), ptr(lse), ptr(g), ptr(dl), N, ncls, ncls, ncls, int(f32),
                  stream_of(lg))
        return dl.to(ctx.in_dtype), None


def cross_entropy(logits, target):
    """Mean-reduced cross entropy (log-softmax + NLL) fused fwd/bwd."""
    if not logits.is_cuda:
        return F.cross_entropy(logits.float(), target)
    return _CrossEntropy.apply(logits, target)


# ================================================================= optimizer
def sgd_flat_(params, grads, momentum_buf, params_bf16, lr, momentum=0.0, dampening=0.0, weight_decay=0.0,
              nesterov=False, first_step=False, grad_scale=1.0):
    """One fused SGD update over flat fp32 buffers (+ bf16 compute-copy refresh)."""
    if not params.is_cuda:
        with torch.no_grad():
            d = grads * grad_scale
            if weight_decay:
                d = d + weight_decay * params
            if momentum:
                if first_step:
                    momentum_buf.copy_(d)
                else:
                    momentum_buf.mul_(momentum).add_(d, alpha=1 - dampening)
                d = d + momentum * momentum_buf if nesterov else momentum_buf
            params.add_(d, alpha=-lr)
            if params_bf16 is not None:
                params_bf16.copy_(params)
        return
    _lib.call("mi_sgd_flat", ptr(params), ptr(grads), ptr(momentum_buf), ptr(params_bf16), params.numel(),
              float(lr), float(momentum), float(dampening), float(weight_decay), int(nesterov), int(first_step),
              float(grad_scale), stream_of(params))


def cast_bf16_(src, dst):
    if not src.is_cuda:
        dst.copy_(src)
        return
    _lib.call("mi_cast_bf16", ptr(src), ptr(dst), src.numel(), stream_of(src))


def checksum(x: torch.Tensor) -> float:
    """Position-weighted fp64 checksum of an fp32 buffer (replica-divergence detector)."""
    if not x.is_cuda:
        idx = (torch.arange(x.numel(), dtype=torch.float64) % 7) + 1
        return float((x.double().reshape(-1) * idx).sum())
    out = torch.empty(1 + 1024, dtype=torch.float64, device=x.device)  # [0] result, [1:] block partials
    _lib.call("mi_checksum", ptr(x), x.numel(), ptr(out), stream_of(x))
    return out[:1]


# ============================================================ input pipeline
_AUG_CONST = {}


def augment(images_u8, out_channels, mean, std, pad=4, flip=True, seed=0, out=None):
    """uint8 NHWC [N,H,W,C] -> bf16 channels_last [N,Cout,H,W]: random crop (zero padding
    ``pad``) + horizontal flip + normalize, all on the GPU (replaces the reference's per-sample
    PIL transforms, cifar10-distributed-smddp-gpu.py:55-62).  ``out``: write into a static
    buffer (the input of a captured HIP-graph step)."""
    N, H, W, C = images_u8.shape
    dev = images_u8.device
    key = (str(dev), max(out_channels, C), C, tuple(mean), tuple(std))
    if key not in _AUG_CONST:  # device constants built once (no per-step host->device copies)
        mean_t = torch.zeros(max(out_channels, C), dtype=torch.float32, device=dev)
        stdinv_t = torch.ones(max(out_channels, C), dtype=torch.float32, device=dev)
        mean_t[:C] = torch.tensor(mean, dtype=torch.float32)
        stdinv_t[:C] = 1.0 / torch.tensor(std, dtype=torch.float32)
        _AUG_CONST[key] = (mean_t, stdinv_t)
    mean_t, stdinv_t = _AUG_CONST[key]
    if not images_u8.is_cuda:
        x = images_u8.float().div(255.0).permute(0, 3, 1, 2)
        x = (x - mean_t[:C].view(1, C, 1, 1)) * stdinv_t[:C].view(1, C, 1, 1)
        return x
    if out is None:
        out = torch.empty((N, out_channels, H, W), dtype=BF16, device=dev, memory_format=CL)
    elif not (out.shape == (N, out_channels, H, W) and out.dtype == BF16 and out.is_contiguous(memory_format=CL)):
        raise ValueError("augment(out=...) needs a bf16 channels_last [N, Cout, H, W] tensor")
    _lib.call("mi_augment", ptr(images_u8.contiguous()), ptr(out), N, H, W, C, out_channels, int(pad), int(flip),
              seed & 0xFFFFFFFF, ptr(mean_t), ptr(stdinv_t), stream_of(images_u8))
    return out
