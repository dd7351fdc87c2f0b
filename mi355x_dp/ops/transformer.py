"""Transformer (ViT-B/16) ops on the native gfx950 kernels.

``encoder_layer`` runs one pre-LN encoder block (torchvision ``EncoderBlock`` semantics:
``y = x + proj(attn(ln_1(x)))``, ``z = y + fc2(gelu(fc1(ln_2(y))))``) as ONE autograd node
with an explicit backward, so every elementwise op rides on a kernel that runs anyway:

  forward                                   backward
  ln_1            mi_layernorm_fwd          dz -> fc2: TN(dW2 + db2), NT+gelu' epilogue -> du
  qkv = h1 Wqkvᵀ  NT (+bias)                du -> fc1: TN(dW1 + db1), NT -> dh2
  attention       attention kernel          dy = dz + ln_2ᵀ(dh2)       (LN bwd, residual add fused)
  y = x + o Woᵀ   NT, residual epilogue     dy -> proj: TN(+bias), NT -> do -> attention bwd -> dqkv
  ln_2            mi_layernorm_fwd          dqkv -> TN(+bias), NT -> dh1
  g = gelu(h2W1ᵀ) NT, GELU epilogue         dx = dy + ln_1ᵀ(dh1)       (LN bwd, residual add fused)
                  (+ gelu' kept for the backward's epilogue, which only multiplies by it)
  z = y + g W2ᵀ   NT, residual epilogue

No torch elementwise kernels, no autograd-inserted residual-gradient adds, and the bias
gradients are column sums of the bf16 gradient computed by the weight-gradient GEMM itself (an
extra MFMA against a ones operand on fragments it already holds -- no second pass over dY).
The data-gradient GEMMs read the flat engine's cached transposed weights.  Weight gradients go
straight into the flat fp32 gradient buffer of the DP engine (``functional._grad_buffer``).

Reference: the ViT-B/16 config is a BASELINE.json target (config 5), not part of the
reference repo; semantics follow torchvision ``vision_transformer.EncoderBlock``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib
from . import kernels as _k  # noqa: F401
from ._lib import ptr, stream_of
from .functional import BF16, _finish_grad, _grad_buffer, _side, linear_weight_t, weight_bf16

F32 = torch.float32
EPI_NONE, EPI_GELU, EPI_GELU_BWD, EPI_RESIDUAL = 0, 1, 2, 3


# ------------------------------------------------------------------ primitives
def _ln_fwd(x2, w, b, eps):
    M, D = x2.shape
    y = torch.empty_like(x2)
    mean = torch.empty(M, dtype=F32, device=x2.device)
    rstd = torch.empty(M, dtype=F32, device=x2.device)
    _lib.call("mi_layernorm_fwd", ptr(x2), ptr(w), ptr(b), ptr(y), ptr(mean), ptr(rstd), M, D, float(eps),
              stream_of(x2))
    return y, mean, rstd


def _ln_bwd(dy2, x2, w, b, mean, rstd, dres=None):
    """dx (+dres), and dW / dB accumulated into the parameters' gradient sinks."""
    M, D = x2.shape
    dx = torch.empty_like(x2)
    gw, gb = _grad_buffer(w), _grad_buffer(b)
    _lib.call("mi_layernorm_bwd", ptr(dy2), ptr(x2), ptr(w), ptr(mean), ptr(rstd), ptr(dres), ptr(dx), ptr(gw),
              ptr(gb), M, D, stream_of(x2))
    return dx, _finish_grad(w, gw), _finish_grad(b, gb)


def _gemm(a2, w16, bias=None, epi=EPI_NONE, aux=None):
    """bf16 out[M][N] = a2[M][K] · w16[N][K]ᵀ (+bias) with the fused epilogue ``epi``."""
    M, K = a2.shape
    N = w16.shape[0]
    out = torch.empty((M, N), dtype=BF16, device=a2.device)
    if epi == EPI_GELU:
        aux = torch.empty((M, N), dtype=BF16, device=a2.device)
    _lib.call("mi_gemm_nt_epi", ptr(a2), ptr(w16), ptr(out), ptr(bias), ptr(aux), epi, M, N, K, K, K, N,
              stream_of(a2))
    return (out, aux) if epi == EPI_GELU else out


def _wbgrad(weight, bias, dy2, x2):
    """weight AND bias gradient from one TN GEMM (the bias column sums ride on its A fragments) --
    on the engine's weight-gradient stream when it has one (functional.WgradStream), overlapping
    the layer's data-gradient chain."""
    g, gb = _grad_buffer(weight), _grad_buffer(bias)
    M, N = dy2.shape
    K = x2.shape[1]

    def launch():
        _lib.call("mi_gemm_tn_bias", ptr(dy2), ptr(x2), ptr(g), ptr(gb), N, K, M, N, K, K, stream_of(dy2))
    side = _side(weight)
    if side is not None and _side(bias) is not None:
        cw, cb = getattr(weight, "_mi_on_grad_ready", None), getattr(bias, "_mi_on_grad_ready", None)

        def ready():
            for c in (cw, cb):
                if c is not None:
                    c()
        side.run(launch, (dy2, x2), ready)
        return None, None
    launch()
    return _finish_grad(weight, g), _finish_grad(bias, gb)


# Plain data-gradient GEMMs (no fused epilogue: the qkv / proj / fc1 input gradients) run on the
# native 256x256 kernel like every other GEMM of the step.  MI355X_DP_BLAS_DGRAD=1 routes them to
# the library GEMM (hipBLASLt) instead: 1.1-1.4x faster on these N = 768 shapes in isolation
# (profiles/vit_r3_gemm_attention.md) but only +1.8 % on the whole ViT-B/16 step
# (profiles/raw/r4_vit_{lib,native}.log: 6,307 vs 6,196 img/s), so the all-native step is the default.
import os as _os
BLAS_DGRAD = _os.environ.get("MI355X_DP_BLAS_DGRAD", "0") == "1"


def _dgrad(dy2, weight, epi=EPI_NONE, aux=None):
    """dX[M][K] = dY[M][N] · W[N][K] (NT against the transposed bf16 weight, cached by the flat
    engine once per optimizer step)."""
    if epi == EPI_NONE and BLAS_DGRAD:
        return torch.matmul(dy2, weight_bf16(weight))
    return _gemm(dy2, linear_weight_t(weight), None, epi, aux)


# ------------------------------------------------------------------ attention
def native_attention_ok(T, head_dim):
    return head_dim == 64 and 0 < T <= 256


_SDPA_WARNED = set()


def _warn_sdpa(T, Dh):
    """The native kernel covers head dim 64 with T <= 256 (ViT-B/16); anything else runs torch's
    scaled_dot_product_attention -- said once per shape, so a non-native path is never silent.
    MI355X_DP_STRICT_NATIVE=1 makes it an error instead."""
    if _os.environ.get("MI355X_DP_STRICT_NATIVE", "0") == "1":
        raise RuntimeError(f"attention: no native kernel for T={T}, head_dim={Dh} (MI355X_DP_STRICT_NATIVE=1)")
    if (T, Dh) not in _SDPA_WARNED:
        _SDPA_WARNED.add((T, Dh))
        import warnings
        warnings.warn(f"mi355x_dp attention: T={T}, head_dim={Dh} is outside the native kernel "
                      f"(head_dim 64, T <= 256); using torch scaled_dot_product_attention", stacklevel=3)


def _attn_fwd(qkv2, B, T, H, need_grad):
    """softmax(q kᵀ/√d) v over the packed [B·T][3·H·Dh] projection; returns o [B·T][H·Dh].
    Native kernel (csrc/kernels/attention.hip) for Dh = 64, T <= 256 (ViT-B/16: T = 197)."""
    D3 = qkv2.shape[1]
    Dh = D3 // (3 * H)
    scale = 1.0 / (Dh ** 0.5)
    if native_attention_ok(T, Dh):
        o = torch.empty((B * T, H * Dh), dtype=BF16, device=qkv2.device)
        lse = torch.empty((B * H * T,), dtype=F32, device=qkv2.device)
        _lib.call("mi_attn_fwd", ptr(qkv2), ptr(o), ptr(lse), B, T, H, float(scale), stream_of(qkv2))
        return o, (("native", lse, o) if need_grad else None)
    _warn_sdpa(T, Dh)
    if not need_grad:
        q, k, v = qkv2.view(B, T, 3, H, Dh).permute(2, 0, 3, 1, 4).unbind(0)
        o4 = F.scaled_dot_product_attention(q, k, v)
        return o4.transpose(1, 2).reshape(B * T, H * Dh), None
    with torch.enable_grad():
        leaf = qkv2.detach().requires_grad_()
        q, k, v = leaf.view(B, T, 3, H, Dh).permute(2, 0, 3, 1, 4).unbind(0)
        o4 = F.scaled_dot_product_attention(q, k, v)
    return o4.detach().transpose(1, 2).reshape(B * T, H * Dh), ("sdpa", leaf, o4)


def _attn_bwd(state, qkv2, do2, B, T, H):
    Dh = do2.shape[1] // H
    if state[0] == "native":
        _, lse, o = state
        dqkv = torch.empty_like(qkv2)
        dvec = torch.empty((B * H * T,), dtype=F32, device=qkv2.device)
        _lib.call("mi_attn_bwd", ptr(qkv2), ptr(o), ptr(do2), ptr(lse), ptr(dvec), ptr(dqkv), B, T, H,
                  float(1.0 / (Dh ** 0.5)), stream_of(qkv2))
        return dqkv
    _, leaf, o4 = state
    (dqkv,) = torch.autograd.grad(o4, leaf, do2.view(B, T, H, Dh).transpose(1, 2))
    return dqkv.contiguous()


def attention(qkv2, B, T, H):
    """Differentiable packed-QKV attention (standalone use / tests)."""
    return _Attention.apply(qkv2, B, T, H)


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv2, B, T, H):
        qkv2 = qkv2.to(BF16).contiguous()
        o, state = _attn_fwd(qkv2, B, T, H, True)
        ctx.state = state
        ctx.dims = (B, T, H)
        ctx.save_for_backward(qkv2)
        return o

    @staticmethod
    def backward(ctx, do):
        (qkv2,) = ctx.saved_tensors
        B, T, H = ctx.dims
        dqkv = _attn_bwd(ctx.state, qkv2, do.to(BF16).contiguous(), B, T, H)
        ctx.state = None
        return dqkv, None, None, None


# ------------------------------------------------------------------ encoder layer
PARAM_ORDER = ("ln_1.weight", "ln_1.bias", "self_attention.in_proj_weight", "self_attention.in_proj_bias",
               "self_attention.out_proj.weight", "self_attention.out_proj.bias", "ln_2.weight", "ln_2.bias",
               "mlp.0.weight", "mlp.0.bias", "mlp.3.weight", "mlp.3.bias")


def _layer_forward(x2, B, T, heads, eps, params, need_grad):
    ln1w, ln1b, wqkv, bqkv, wo, bo, ln2w, ln2b, w1, b1, w2, b2 = params
    h1, m1, r1 = _ln_fwd(x2, ln1w, ln1b, eps)
    qkv = _gemm(h1, weight_bf16(wqkv), bqkv)
    o, attn = _attn_fwd(qkv, B, T, heads, need_grad)
    y = _gemm(o, weight_bf16(wo), bo, EPI_RESIDUAL, x2)
    h2, m2, r2 = _ln_fwd(y, ln2w, ln2b, eps)
    g, u = _gemm(h2, weight_bf16(w1), b1, EPI_GELU)  # u = gelu'(pre-activation): all the backward needs
    z = _gemm(g, weight_bf16(w2), b2, EPI_RESIDUAL, y)
    saved = (x2, h1, m1, r1, qkv, o, y, h2, m2, r2, u, g) if need_grad else None
    return z, saved, attn


class _EncoderLayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, heads, eps, *params):
        B, T, D = x.shape
        x2 = x.reshape(B * T, D)
        if x2.dtype != BF16:
            x2 = x2.to(BF16)
        x2 = x2.contiguous()
        z, saved, attn = _layer_forward(x2, B, T, heads, eps, params, True)
        ctx.save_for_backward(*saved, *params)
        ctx.attn = attn
        ctx.dims = (B, T, D, heads)
        ctx.in_dtype = x.dtype
        return z.view(B, T, D)

    @staticmethod
    def backward(ctx, dz):
        B, T, D, heads = ctx.dims
        (x2, h1, m1, r1, qkv, o, y, h2, m2, r2, u, g, ln1w, ln1b, wqkv, bqkv, wo, bo, ln2w, ln2b, w1, b1, w2,
         b2) = ctx.saved_tensors
        dz2 = dz.reshape(B * T, D)
        if dz2.dtype != BF16:
            dz2 = dz2.to(BF16)
        dz2 = dz2.contiguous()
        # MLP
        d_w2, d_b2 = _wbgrad(w2, b2, dz2, g)
        du = _dgrad(dz2, w2, EPI_GELU_BWD, u)
        d_w1, d_b1 = _wbgrad(w1, b1, du, h2)
        dh2 = _dgrad(du, w1)
        dy, d_ln2w, d_ln2b = _ln_bwd(dh2, y, ln2w, ln2b, m2, r2, dres=dz2)
        # attention
        d_wo, d_bo = _wbgrad(wo, bo, dy, o)
        do = _dgrad(dy, wo)
        dqkv = _attn_bwd(ctx.attn, qkv, do, B, T, heads)
        ctx.attn = None
        d_wqkv, d_bqkv = _wbgrad(wqkv, bqkv, dqkv, h1)
        dh1 = _dgrad(dqkv, wqkv)
        dx, d_ln1w, d_ln1b = _ln_bwd(dh1, x2, ln1w, ln1b, m1, r1, dres=dy)
        dx = dx.view(B, T, D)
        if ctx.in_dtype != BF16:
            dx = dx.to(ctx.in_dtype)
        return (dx, None, None, d_ln1w, d_ln1b, d_wqkv, d_bqkv, d_wo, d_bo, d_ln2w, d_ln2b, d_w1, d_b1, d_w2,
                d_b2)


def encoder_layer(x, heads, eps, params):
    """x [B, T, D] (cuda) -> [B, T, D] bf16.  ``params`` in ``PARAM_ORDER``."""
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
        return _EncoderLayer.apply(x, heads, eps, *params)
    B, T, D = x.shape
    x2 = x.reshape(B * T, D).to(BF16).contiguous()
    z, _, _ = _layer_forward(x2, B, T, heads, eps, params, False)
    return z.view(B, T, D)


# ------------------------------------------------------------------ standalone LayerNorm
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if x2.dtype != BF16:
            x2 = x2.to(BF16)
        x2 = x2.contiguous()
        y, mean, rstd = _ln_fwd(x2, w, b, eps)
        ctx.save_for_backward(x2, w, b, mean, rstd)
        ctx.shape = shape
        ctx.in_dtype = x.dtype
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, b, mean, rstd = ctx.saved_tensors
        dy2 = dy.reshape(x2.shape)
        if dy2.dtype != BF16:
            dy2 = dy2.to(BF16)
        dx, dw, db = _ln_bwd(dy2.contiguous(), x2, w, b, mean, rstd)
        dx = dx.view(ctx.shape)
        if ctx.in_dtype != BF16:
            dx = dx.to(ctx.in_dtype)
        return dx, dw, db, None


class _PatchEmbed(torch.autograd.Function):
    """Stride = kernel = p patch embedding as patchify + one plain GEMM: the NHWC input's real
    channels C are gathered into [patches][p * p * C] rows in (r, s, c) order -- the flat engine's
    [K][R][S][C] conv weight layout, so the weight and its gradient are used as [K][p * p * C]
    matrices in place -- instead of the 8-channel-padded implicit-GEMM conv (K = 768 instead of 2048
    for ViT-B/16).  Returns [N][patches][K] bf16; no input gradient (images)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        N, Cs, H, W = x.shape
        K, C, R, S = weight.shape
        Kd = R * S * C
        rows = N * (H // R) * (W // S)
        st = stream_of(x)
        xp = torch.empty((rows, Kd), dtype=BF16, device=x.device)
        _lib.call("mi_vit_patchify", ptr(x), ptr(xp), N, H, W, Cs, C, R, st)
        w2 = weight_bf16(weight).permute(0, 2, 3, 1)
        w2 = w2.reshape(K, Kd) if w2.is_contiguous() else w2.contiguous().reshape(K, Kd)
        y = torch.empty((rows, K), dtype=BF16, device=x.device)
        _lib.call("mi_gemm_nt", ptr(xp), ptr(w2), ptr(y), ptr(bias), ptr(None), rows, K, Kd, Kd, Kd, K, 0, 0, st)
        ctx.save_for_backward(xp)
        ctx.params = (weight, bias)
        return y.view(N, rows // N, K)

    @staticmethod
    def backward(ctx, dy):
        (xp,) = ctx.saved_tensors
        weight, bias = ctx.params
        rows, Kd = xp.shape
        K = weight.shape[0]
        dy2 = dy.reshape(rows, K).to(BF16).contiguous()
        st = stream_of(dy2)
        dw = db = None
        if ctx.needs_input_grad[1]:
            g = _grad_buffer(weight)
            g2 = g.permute(0, 2, 3, 1)  # [K][R][S][C]: contiguous in the kernel layout
            tmp = None if g2.is_contiguous() else torch.zeros(g2.shape, dtype=F32, device=g.device)
            _lib.call("mi_gemm_tn", ptr(dy2), ptr(xp), ptr(g2 if tmp is None else tmp), K, Kd, rows, K, Kd, Kd, st)
            if tmp is not None:
                g2.add_(tmp)
            dw = _finish_grad(weight, g)
        if bias is not None and ctx.needs_input_grad[2]:
            gb = _grad_buffer(bias)
            _lib.call("mi_colsum_bf16", ptr(dy2), ptr(gb), rows, K, K, st)
            db = _finish_grad(bias, gb)
        return None, dw, db


def patch_embed_ok(x, conv) -> bool:
    K, C, R, S = conv.weight.shape
    return (x.is_cuda and x.dtype == BF16 and x.is_contiguous(memory_format=torch.channels_last)
            and tuple(conv.stride) == (R, S) and R == S and tuple(conv.padding) == (0, 0) and conv.groups == 1
            and C <= x.shape[1] and (R * S * C) % 8 == 0 and K % 8 == 0 and x.shape[2] % R == 0
            and x.shape[3] % S == 0 and conv.weight.dtype == torch.float32)


def patch_embed(x, conv):
    """[N][patches][K] bf16 embedding of the NHWC bf16 image batch ``x`` by the stride-p conv ``conv``."""
    return _PatchEmbed.apply(x, conv.weight, conv.bias)


class _VitEmbed(torch.autograd.Function):
    """[class token ; patch embeddings] + position embedding as one native pass
    (``mi_vit_embed_fwd``); backward: the patches' dense gradient plus the fixed-order batch sums
    for the position embedding and the class token (``mi_vit_embed_bwd``) -- no concatenation,
    broadcast-add, cast or reduction launches."""

    @staticmethod
    def forward(ctx, patches, cls, pos):
        N, P, D = patches.shape
        T = P + 1
        p = patches.contiguous()
        out = torch.empty((N, T, D), dtype=BF16, device=p.device)
        _lib.call("mi_vit_embed_fwd", ptr(p), ptr(cls), ptr(pos), ptr(out), N, T, D, stream_of(p))
        ctx.params = (cls, pos)
        ctx.shape = (N, T, D)
        return out

    @staticmethod
    def backward(ctx, dout):
        cls, pos = ctx.params
        N, T, D = ctx.shape
        d = dout.to(BF16).contiguous()
        dp = torch.empty((N, T - 1, D), dtype=BF16, device=d.device)
        gpos = _grad_buffer(pos) if ctx.needs_input_grad[2] else None
        gcls = _grad_buffer(cls) if ctx.needs_input_grad[1] else None
        part = torch.empty(int(_lib.load().mi_vit_embed_bwd_part_floats(N, T, D)), dtype=F32, device=d.device)
        _lib.call("mi_vit_embed_bwd", ptr(d), ptr(dp), ptr(gpos), ptr(gcls), ptr(part), N, T, D, stream_of(d))
        dcls = _finish_grad(cls, gcls) if gcls is not None else None
        dpos = _finish_grad(pos, gpos) if gpos is not None else None
        return dp, dcls, dpos


def vit_embed(patches, cls, pos):
    """bf16 [N][T][D] tokens = cat(cls, patches) + pos for fp32 ``cls`` [1,1,D] / ``pos`` [1,T,D]."""
    return _VitEmbed.apply(patches, cls, pos)


def layer_norm(x, weight, bias, eps):
    """Native LayerNorm over the last dim (bf16 out, fp32 affine parameters)."""
    return _LayerNorm.apply(x, weight, bias, eps)
