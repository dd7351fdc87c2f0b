"""ResNet stem (conv1 7x7/2 -> bn1 -> relu -> maxpool 3x3/2) as ONE autograd node.

The stem's BN/ReLU output (64 x 112 x 112 per image, 411 MB at batch 256) is the largest
activation of ResNet-50 and its only consumer is the max pool.  The per-op chain writes it, reads
it back for the pool, and in backward reads it twice more (maxpool arg-max routing, ReLU mask)
while materialising two full-resolution gradients.  Here:

  forward : small-channel MFMA conv (epilogue emits BN statistics) -> BN finalize only ->
            ``bnpool_fwd``: pool(relu(c*scale + shift)) straight from the conv output c, plus
            the uint8 arg-max tap; the full-resolution activation is never stored;
  backward: ``bnpool_bwd``: per input pixel, gather dpool through the arg-max, recompute the
            ReLU mask from c, reduce the BN backward statistics (pass 1), regather and write
            dc = BN-backward(dz) (pass 2) -> conv weight gradient (c8 TN kernel).

Reference: torchvision ResNet stem reached through ``torchvision.models.resnet18``
(cifar10-distributed-smddp-gpu.py:30-32); the same semantics as the unfused
``conv_bn(conv1, bn1, relu=True)`` + ``MaxPool2d(3, 2, 1)`` path (same arg-max tie rule).
"""
from __future__ import annotations

import torch

from . import _lib
from . import kernels as _k  # noqa: F401
from ._lib import ptr, stream_of
from .functional import BF16, CL, _finish_grad, _grad_buffer, _nhwc, pad_channels8, weight_bf16

F32 = torch.float32


def _out(h, r, s, p):
    return (h + 2 * p - r) // s + 1


class _Stem(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, geom, wconv, gamma, beta, rmean, rvar, nbt, momentum, eps):
        stride, pad, pk, ps, pp = geom
        N, C, H, W = x.shape
        K, Cw, R, S = wconv.shape
        P, Q = _out(H, R, stride, pad), _out(W, S, stride, pad)
        P2, Q2 = _out(P, pk, ps, pp), _out(Q, pk, ps, pp)
        dev = x.device
        st = stream_of(x)
        lib = _lib.load()
        # conv: small-channel (8-wide tap) MFMA mode, BN statistics from the epilogue
        w16 = weight_bf16(wconv)
        wp = torch.empty((K, R, S, 8), dtype=BF16, device=dev)  # zero-padded to 8 channels, one launch
        _lib.call("mi_stem_wpack", ptr(w16), ptr(wp), K, Cw, R, S, *w16.stride(), st)
        rows = lib.mi_conv_stat_rows_g(N, H, W, 8, K, R, S, stride, pad, P, Q)
        slab = torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, K), dtype=F32, device=dev)
        c = torch.empty((N, K, P, Q), dtype=BF16, device=dev, memory_format=CL)
        _lib.call("mi_conv2d_fwd", ptr(x), ptr(wp), ptr(c), ptr(None), ptr(slab), N, H, W, 8, K, R, S, stride, pad,
                  P, Q, 0, st)
        f32 = dict(dtype=F32, device=dev)
        mean, invstd = torch.empty(K, **f32), torch.empty(K, **f32)
        scale, shift = torch.empty(K, **f32), torch.empty(K, **f32)
        _lib.call("mi_bn_fwd_train", ptr(c), ptr(None), ptr(None), N * P * Q, K, float(eps), float(momentum),
                  ptr(gamma), ptr(beta), ptr(rmean), ptr(rvar), ptr(nbt), ptr(mean), ptr(invstd), ptr(scale),
                  ptr(shift), ptr(slab), int(rows), 1, st)
        y = torch.empty((N, K, P2, Q2), dtype=BF16, device=dev, memory_format=CL)
        idx = torch.empty((N, P2, Q2, K), dtype=torch.uint8, device=dev)
        _lib.call("mi_bnpool_fwd", ptr(c), ptr(scale), ptr(shift), ptr(y), ptr(idx), N, P, Q, K, P2, Q2, pk, ps, pp,
                  st)
        ctx.save_for_backward(x, c, idx, mean, invstd, scale, shift)
        ctx.params = (wconv, gamma, beta)
        ctx.geom = (N, H, W, K, Cw, R, S, stride, pad, P, Q, P2, Q2, pk, ps, pp)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, c, idx, mean, invstd, scale, shift = ctx.saved_tensors
        wconv, gamma, beta = ctx.params
        N, H, W, K, Cw, R, S, stride, pad, P, Q, P2, Q2, pk, ps, pp = ctx.geom
        dy = _nhwc(dy)
        dev = dy.device
        st = stream_of(dy)
        lib = _lib.load()
        gw, gb = _grad_buffer(gamma), _grad_buffer(beta)
        M = N * P * Q
        # the k3/s2/p1 pass reduces over output-pixel quads, the generic one over input pixels
        rows = max(lib.mi_bnpool_partial_rows(M, K), lib.mi_bnpool_partial_rows(N * P2 * Q2, K))
        part = torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, K), dtype=F32, device=dev)
        coef = torch.empty((3, K), dtype=F32, device=dev)
        dc = torch.empty_like(c, memory_format=CL)
        _lib.call("mi_bnpool_bwd", ptr(dy), ptr(idx), ptr(c), ptr(dc), N, P, Q, K, P2, Q2, pk, ps, pp, ptr(scale),
                  ptr(shift), ptr(gamma), ptr(mean), ptr(invstd), ptr(gw), ptr(gb), ptr(coef), ptr(part), st)
        dgamma, dbeta = _finish_grad(gamma, gw), _finish_grad(beta, gb)
        g = _grad_buffer(wconv)
        # the persistent stem kernel's fixed-order partial sums land in g's own layout; otherwise
        # (other geometry, atomic mode) a padded buffer is cropped and permuted into g
        rc = lib.mi_stem_wgrad_to(ptr(x), ptr(dc), ptr(g), Cw, *g.stride(), N, H, W, K, R, S, stride, P, Q, pad, st)
        if rc != 0:
            gp = torch.zeros((K, R, S, 8), dtype=F32, device=dev)
            _lib.call("mi_conv2d_wgrad", ptr(x), ptr(dc), ptr(gp), N, H, W, 8, K, R, S, stride, pad, P, Q, st)
            g.add_(gp[..., :Cw].permute(0, 3, 1, 2))
        dw = _finish_grad(wconv, g)
        return None, None, dw, dgamma, dbeta, None, None, None, None, None


def fusable(conv, bn, pool, x) -> bool:
    """CUDA training step with a small-channel stem conv (C <= 8, bias-free), a batch-statistics
    BN with running stats and fixed momentum, a plain max pool, and an input that needs no
    gradient (the stem dgrad is never needed for images)."""
    from mi355x_dp.models.layers import BatchNorm2d, Conv2d, MaxPool2d
    if not (x.is_cuda and x.dtype == BF16 and torch.is_grad_enabled() and bn.training and not x.requires_grad):
        return False
    if not (isinstance(conv, Conv2d) and isinstance(bn, BatchNorm2d) and isinstance(pool, MaxPool2d)):
        return False
    if conv.bias is not None or conv.groups != 1 or conv.in_channels > 8 or conv.out_channels % 8 != 0:
        return False
    if len(set(conv.stride)) != 1 or len(set(conv.padding)) != 1 or conv.dilation not in ((1, 1), 1):
        return False
    if not bn.track_running_stats or not bn.affine or bn.momentum is None:
        return False
    ks = pool.kernel_size if isinstance(pool.kernel_size, int) else pool.kernel_size[0]
    if pool.ceil_mode or pool.dilation not in (1, (1, 1)) or ks * ks > 255:
        return False
    return True


def stem(conv, bn, pool, x):
    """maxpool(relu(bn(conv(x)))) as one fused node (caller checked ``fusable``)."""
    def _i(v):
        return int(v if isinstance(v, int) else v[0])
    if x.shape[1] != 8 or x.dtype != BF16 or not x.is_contiguous(memory_format=CL):
        x = pad_channels8(x) if x.shape[1] < 8 else _nhwc(x)
    geom = (_i(conv.stride), _i(conv.padding), _i(pool.kernel_size), _i(pool.stride), _i(pool.padding))
    return _Stem.apply(x, geom, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                       bn.num_batches_tracked, float(bn.momentum), float(bn.eps))
