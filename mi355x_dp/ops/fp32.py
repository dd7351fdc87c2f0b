"""fp32 compute mode (``MI355X_DP_COMPUTE_DTYPE=fp32``): the ResNet training path on native fp32
kernels (csrc/kernels/fp32.hip: ``v_mfma_f32_16x16x4_f32`` implicit-GEMM convolutions, fp32
BatchNorm / pooling / Linear), so the reference workload -- fp32 on A100,
cifar10-distributed-smddp-gpu.py:145-158 -- can be compared like for like.
gfx950 has no TF32: these are exact fp32 products with fp32 accumulation.

Device contract: fp32 activations in ``channels_last`` (NHWC storage), channel counts a multiple
of 4 (the 3-channel image input is zero-padded to 4); conv weights read in ``[K][R][S][C]`` order
(the flat engine's master layout, used in place).  Gradients go into the flat engine's fp32 buffer
through the same sinks as the bf16 path (``functional._grad_buffer`` / ``_finish_grad``: the
engine's ready-marks and bucket collectives are unchanged).  Deterministic: split-K partials are
summed in split order, BatchNorm reductions in block order in fp64, max-pool backward is a gather.
"""
from __future__ import annotations

import os

import torch

from . import _lib
from . import kernels as _k  # noqa: F401  (registers signatures)
from ._lib import ptr, stream_of
from .functional import _finish_grad, _grad_buffer

F32 = torch.float32
CL = torch.channels_last
COMPUTE_FP32 = os.environ.get("MI355X_DP_COMPUTE_DTYPE", "bf16").lower() in ("fp32", "float32")


def active(x: torch.Tensor) -> bool:
    """is ``x`` an activation of the fp32 compute mode?"""
    return COMPUTE_FP32 and x.is_cuda and x.dtype == F32


def _out(h, r, s, p):
    return (h + 2 * p - r) // s + 1


def _nhwc(x):
    if x.dtype != F32:
        x = x.float()
    return x if x.is_contiguous(memory_format=CL) else x.contiguous(memory_format=CL)


def to_input(x: torch.Tensor) -> torch.Tensor:
    """model entry: fp32 NHWC, channels zero-padded to a multiple of 4"""
    N, C, H, W = x.shape
    Cp = (C + 3) // 4 * 4
    if Cp == C:
        return _nhwc(x)
    out = torch.empty((N, Cp, H, W), dtype=F32, device=x.device, memory_format=CL)
    out[:, C:].zero_()
    out[:, :C].copy_(x)
    return out


def _weight_krsc(w: torch.Tensor, C: int) -> torch.Tensor:
    """[K][R][S][C] fp32 operand of a [K, Cw, R, S] weight (zero-padded to C input channels)"""
    K, Cw, R, S = w.shape
    if Cw == C and w.dtype == F32 and w.is_contiguous(memory_format=CL):
        return w  # the flat engine's master weight, in place
    out = torch.zeros((K, R, S, C), dtype=F32, device=w.device)
    out[..., :Cw].copy_(w.detach().permute(0, 2, 3, 1))
    return out


def _conv(mode, a, b, out, accumulate, geom, bias=None):
    Nb, H, W, C, K, R, S, stride, pad, P, Q = geom
    lib = _lib.load()
    n = lib.mi_f32_conv_ws_floats(mode, Nb, H, W, C, K, R, S, stride, pad, P, Q)
    ws = torch.empty(n, dtype=F32, device=out.device) if n else None
    _lib.call("mi_f32_conv", mode, ptr(a), ptr(b), ptr(out), ptr(ws), ptr(bias), int(accumulate), Nb, H, W, C, K, R,
              S, stride, pad, P, Q, stream_of(out))


class _ConvF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad):
        x = to_input(x) if x.shape[1] % 4 else _nhwc(x)
        N, C, H, W = x.shape
        K, Cw, R, S = weight.shape
        P, Q = _out(H, R, stride, pad), _out(W, S, stride, pad)
        wk = _weight_krsc(weight, C)
        y = torch.empty((N, K, P, Q), dtype=F32, device=x.device, memory_format=CL)
        b = bias.detach().float().contiguous() if bias is not None else None
        _conv(0, x, wk, y, 0, (N, H, W, C, K, R, S, stride, pad, P, Q), b)
        ctx.save_for_backward(x, weight, wk)
        ctx.geom = (N, H, W, C, K, R, S, stride, pad, P, Q)
        ctx.bias = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, wk = ctx.saved_tensors
        N, H, W, C, K, R, S, stride, pad, P, Q = geom = ctx.geom
        dy = _nhwc(dy)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((N, C, H, W), dtype=F32, device=dy.device, memory_format=CL)
            _conv(1, dy, wk, dx, 0, geom)
            if C != weight.shape[1]:
                dx = dx[:, :weight.shape[1]]
        if ctx.needs_input_grad[1]:
            g = _grad_buffer(weight)
            if C == weight.shape[1] and g.is_contiguous(memory_format=CL):
                _conv(2, dy, x, g, 1, geom)  # accumulate straight into the [K][R][S][C] sink
            else:
                gp = torch.zeros((K, R, S, C), dtype=F32, device=dy.device)
                _conv(2, dy, x, gp, 0, geom)
                g.add_(gp[..., :weight.shape[1]].permute(0, 3, 1, 2))
            dw = _finish_grad(weight, g)
        if ctx.bias is not None and ctx.needs_input_grad[2]:
            gb = _grad_buffer(ctx.bias)
            _lib.call("mi_f32_colsum", ptr(dy), ptr(gb), N * P * Q, K, 1, stream_of(dy))
            db = _finish_grad(ctx.bias, gb)
        return dx, dw, db, None, None


def conv2d(x, weight, bias=None, stride=1, padding=0):
    return _ConvF32.apply(x, weight, bias, int(stride), int(padding))


class _BNF32(torch.autograd.Function):
    """training-mode BatchNorm2d with fused residual add and ReLU: y = act(bn(x) (+ res))"""

    @staticmethod
    def forward(ctx, x, gamma, beta, res, rmean, rvar, nbt, momentum, eps, relu):
        x = _nhwc(x)
        N, C, H, W = x.shape
        M = N * H * W
        lib = _lib.load()
        dev = x.device
        part = torch.empty((lib.mi_f32_bn_partial_rows(M, C), 2, C), dtype=F32, device=dev)
        mean, invstd, scale, shift = (torch.empty(C, dtype=F32, device=dev) for _ in range(4))
        y = torch.empty_like(x, memory_format=CL)
        r = _nhwc(res) if res is not None else None
        _lib.call("mi_f32_bn_fwd_train", ptr(x), ptr(r), ptr(y), M, C, float(eps), float(momentum), ptr(gamma),
                  ptr(beta), ptr(rmean), ptr(rvar), ptr(nbt), ptr(mean), ptr(invstd), ptr(scale), ptr(shift),
                  ptr(part), int(relu), stream_of(x))
        ctx.save_for_backward(x, y, gamma, mean, invstd)
        ctx.params = (gamma, beta)
        ctx.relu, ctx.has_res = bool(relu), res is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, gamma, mean, invstd = ctx.saved_tensors
        g_param, b_param = ctx.params
        dy = _nhwc(dy)
        N, C, H, W = x.shape
        M = N * H * W
        lib = _lib.load()
        dev = dy.device
        part = torch.empty((lib.mi_f32_bn_partial_rows(M, C), 2, C), dtype=F32, device=dev)
        coef = torch.empty((3, C), dtype=F32, device=dev)
        dx = torch.empty_like(x, memory_format=CL)
        dres = torch.empty_like(x, memory_format=CL) if ctx.has_res else None
        gw = _grad_buffer(g_param) if g_param is not None else None
        gb = _grad_buffer(b_param) if b_param is not None else None
        _lib.call("mi_f32_bn_bwd_train", ptr(dy), ptr(y), ptr(x), ptr(dx), ptr(dres), M, C, ptr(gamma), ptr(mean),
                  ptr(invstd), ptr(gw), ptr(gb), ptr(coef), ptr(part), int(ctx.relu), stream_of(dy))
        dgw = _finish_grad(g_param, gw) if gw is not None else None
        dgb = _finish_grad(b_param, gb) if gb is not None else None
        return dx, dgw, dgb, dres, None, None, None, None, None, None


def batch_norm_act(x, weight, bias, running_mean, running_var, num_batches_tracked, training, momentum, eps,
                   relu=False, residual=None):
    if training:
        return _BNF32.apply(x, weight, bias, residual, running_mean, running_var, num_batches_tracked, momentum, eps,
                            relu)
    # eval: per-channel affine from the running statistics (a few tiny tensor ops), one native pass
    x = _nhwc(x)
    N, C, H, W = x.shape
    with torch.no_grad():
        inv = torch.rsqrt(running_var.float() + eps)
        scale = (weight.float() * inv) if weight is not None else inv
        shift = (bias.float() if bias is not None else 0.0) - running_mean.float() * scale
        scale, shift = scale.contiguous(), shift.contiguous()
    y = torch.empty_like(x, memory_format=CL)
    r = _nhwc(residual) if residual is not None else None
    _lib.call("mi_f32_bn_apply", ptr(x), ptr(r), ptr(y), N * H * W, C, ptr(scale), ptr(shift), int(relu),
              stream_of(x))
    return y


class _MaxPoolF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        x = _nhwc(x)
        N, C, H, W = x.shape
        P, Q = _out(H, k, s, pad), _out(W, k, s, pad)
        y = torch.empty((N, C, P, Q), dtype=F32, device=x.device, memory_format=CL)
        tap = torch.empty((N, P, Q, C), dtype=torch.uint8, device=x.device)
        _lib.call("mi_f32_maxpool_fwd", ptr(x), ptr(y), ptr(tap), N, H, W, C, P, Q, k, s, pad, stream_of(x))
        ctx.save_for_backward(tap)
        ctx.geom = (N, C, H, W, P, Q, k, s, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (tap,) = ctx.saved_tensors
        N, C, H, W, P, Q, k, s, pad = ctx.geom
        dy = _nhwc(dy)
        dx = torch.empty((N, C, H, W), dtype=F32, device=dy.device, memory_format=CL)
        _lib.call("mi_f32_maxpool_bwd", ptr(dy), ptr(tap), ptr(dx), N, H, W, C, P, Q, k, s, pad, stream_of(dy))
        return dx, None, None, None


def max_pool2d(x, k=3, s=2, pad=1):
    return _MaxPoolF32.apply(x, int(k), int(s), int(pad))


class _GapF32(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _nhwc(x)
        N, C, H, W = x.shape
        y = torch.empty((N, C), dtype=F32, device=x.device)
        _lib.call("mi_f32_gap_fwd", ptr(x), ptr(y), N, H * W, C, stream_of(x))
        ctx.geom = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.geom
        dy = dy.float().contiguous()
        dx = torch.empty((N, C, H, W), dtype=F32, device=dy.device, memory_format=CL)
        _lib.call("mi_f32_gap_bwd", ptr(dy), ptr(dx), N, H * W, C, stream_of(dy))
        return dx


def global_avg_pool(x):
    return _GapF32.apply(x)


class _LinearF32(torch.autograd.Function):
    """y = x W^T + b as a 1x1 convolution of [M, 1, 1, in] rows (the same fp32 MFMA kernel)"""

    @staticmethod
    def forward(ctx, x, weight, bias):
        x2 = x.reshape(-1, x.shape[-1]).float().contiguous()
        M, Kd = x2.shape
        N = weight.shape[0]
        if Kd % 4 or N % 4:
            raise NotImplementedError("fp32 native linear needs in / out features % 4 == 0")
        w = weight if weight.dtype == F32 and weight.is_contiguous() else weight.detach().float().contiguous()
        y = torch.empty((M, N), dtype=F32, device=x.device)
        b = bias.detach().float().contiguous() if bias is not None else None
        _conv(0, x2, w, y, 0, (M, 1, 1, Kd, N, 1, 1, 1, 0, 1, 1), b)
        ctx.save_for_backward(x2, weight, w)
        ctx.bias = bias
        ctx.in_shape = x.shape
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, w = ctx.saved_tensors
        M, Kd = x2.shape
        N = weight.shape[0]
        dy2 = dy.reshape(M, N).float().contiguous()
        geom = (M, 1, 1, Kd, N, 1, 1, 1, 0, 1, 1)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dxf = torch.empty((M, Kd), dtype=F32, device=dy.device)
            _conv(1, dy2, w, dxf, 0, geom)
            dx = dxf.reshape(ctx.in_shape)
        if ctx.needs_input_grad[1]:
            g = _grad_buffer(weight)
            if g.is_contiguous():
                _conv(2, dy2, x2, g, 1, geom)
            else:
                gp = torch.zeros((N, Kd), dtype=F32, device=dy.device)
                _conv(2, dy2, x2, gp, 0, geom)
                g.add_(gp)
            dw = _finish_grad(weight, g)
        if ctx.bias is not None and ctx.needs_input_grad[2]:
            gb = _grad_buffer(ctx.bias)
            _lib.call("mi_f32_colsum", ptr(dy2), ptr(gb), M, N, 1, stream_of(dy2))
            db = _finish_grad(ctx.bias, gb)
        return dx, dw, db


def linear(x, weight, bias=None):
    return _LinearF32.apply(x, weight, bias)


__all__ = ["COMPUTE_FP32", "active", "to_input", "conv2d", "batch_norm_act", "max_pool2d", "global_avg_pool",
           "linear"]
