"""ResNet residual blocks (torchvision BasicBlock / Bottleneck) as ONE autograd node each.

Per-op autograd (conv -> BN -> ...) leaves two kinds of memory traffic on the table in the
backward pass, which at ResNet-50 / batch 256 is bandwidth-bound outside the convolutions:

* the gradient of a block input is a SUM (conv1's data gradient + the residual path); autograd
  materialises both and adds them with a separate elementwise kernel;
* every BatchNorm backward re-reads dy, y and x once for its statistics pass and once more for
  its apply pass.

With the block as one node the backward is scheduled explicitly:

  bn3 backward (relu mask + residual): dres is written straight into the block's dx buffer
  (identity shortcut) or the downsample BN's gradient;
  conv3 dgrad with epilogue 4: emits dz2 = dgrad * [y2 > 0] AND bn2's backward statistics
  (sum dz2, sum dz2 * (c2 - mean2)) from the same registers -> bn2 needs no statistics pass
  and its apply pass reads dz2, c2 only (no y2);
  conv2 dgrad with epilogue 4 for bn1 likewise;
  conv1 (and downsample) dgrad with epilogue 3: accumulate into dx in place -- no add kernel;
  when the block input is the previous block's output, epilogue 5 instead: accumulate, then
  the previous block's final relu mask + its last-BN backward statistics, handed over so the
  previous block skips its statistics pass and uses the buffer as its residual gradient.

Forward is the per-op kernel sequence (conv epilogue emits the BN forward statistics, BN apply
fuses residual + ReLU), except that a projection shortcut's BatchNorm is applied inside the last
BN's pass (``mi_bn_apply_dual``) instead of being written out and re-read as the residual.  Weight gradients go into the flat fp32 gradient
buffer of the DP engine.  Reference: torchvision BasicBlock / Bottleneck semantics, reached by
the reference through ``torchvision.models.resnet18`` (cifar10-distributed-smddp-gpu.py:30-32).
"""
from __future__ import annotations

import os

import torch

from . import _lib
from . import kernels as _k  # noqa: F401
from ._lib import ptr, stream_of
from .functional import BF16, CL, _finish_grad, _grad_buffer, _nhwc, _side, run_wgrad, weight_bf16, weight_bf16_t

F32 = torch.float32
EPI_ACCUM, EPI_BN_BWD, EPI_ACCUM_BN_BWD = 3, 4, 5
# mi_conv2d_dgrad_ex2 flags: write only the parity classes some tap reaches (stride 2) / read the
# accumulated-into gradient only at even (h, w)
DGRAD_SPARSE, DGRAD_ACC_EVEN = 1, 2

# Cross-block hand-off: the dgrad that completes block k+1's input gradient (residual sum) also
# applies block k's final relu mask and emits block k's last-BN backward statistics (epilogue 5).
# The statistics are parked here keyed by the gradient buffer; block k's backward takes them
# only if it receives that very buffer unmodified (same storage, same version) -- otherwise
# it runs its own statistics pass, which is still correct because re-masking is idempotent.
_HANDOFF = {}
HANDOFF_USED = [0]  # diagnostics: backward passes that consumed a hand-off


# The projection shortcut (downsample conv + BN) of a stage's first block is independent of the
# main conv1 -> conv2 -> conv3 chain until the final sum: it runs on an auxiliary stream, forward
# (conv + BN statistics / finalize) and backward (BN backward + data gradient into dx), joined
# just before the consumer.  Opt-in (MI355X_DP_DS_STREAM=1): on ResNet-50 bs256 it measured 12.41k
# vs 12.47k img/s -- the branch is too small to pay for the third stream's contention.
DS_STREAM = os.environ.get("MI355X_DP_DS_STREAM", "0") == "1"
_AUX_STREAMS = {}


def _aux_stream(dev):
    from .functional import WgradStream
    if not DS_STREAM or dev.type != "cuda" or WgradStream.suspended or torch.cuda.is_current_stream_capturing():
        return None
    s = _AUX_STREAMS.get(dev.index)
    if s is None:
        s = _AUX_STREAMS[dev.index] = torch.cuda.Stream(device=dev)
        # its own split-K slab workspace: with the weight-gradient stream off, the shortcut's weight
        # gradient on this stream runs concurrently with the compute stream's split-K TN kernels
        from . import _lib
        import ctypes
        with torch.cuda.device(dev):
            _lib.call("mi_register_aux_stream", ctypes.c_void_p(s.cuda_stream))
    return s


def _out_hw(h, r, stride, pad):
    return (h + 2 * pad - r) // stride + 1


class _ConvSpec:
    __slots__ = ("w", "stride", "pad")

    def __init__(self, conv):
        self.w = conv.weight
        self.stride = int(conv.stride[0])
        self.pad = int(conv.padding[0])


class _BNSpec:
    __slots__ = ("w", "b", "rm", "rv", "nbt", "momentum", "eps")

    def __init__(self, bn):
        self.w, self.b = bn.weight, bn.bias
        self.rm, self.rv, self.nbt = bn.running_mean, bn.running_var, bn.num_batches_tracked
        self.momentum = float(bn.momentum)
        self.eps = float(bn.eps)


# Normalize-on-load of the inner BatchNorms (bn1 / bn2 of a bottleneck, bn1 of a basic block): the
# conv that consumes an inner BN's output reads the raw conv output c and applies relu(c * scale +
# shift) as it stages its operand (forward and weight gradient), and the data gradient that needs
# that BN's ReLU mask takes it from c -- the BN output y is never written nor read (VERDICT r3
# item 2; profiles/bn_nol_r4.md).  Per consumer shape, where the 128-tile kernels serve all three
# (mi_conv_nol_ok); elsewhere y is materialised as before.  OFF by default (MI355X_DP_NOL=1 enables):
# on MI355X the in-kernel transform costs more than the bn_apply pass it removes -- every NoL kernel
# is slower in isolation (fwd +10-30 %, mask-from-c dgrad +2-10 %, wgrad +1-65 %,
# tools/bench_nol.py) and the RN50 bs256 step loses ~1 % (same-box A/B, profiles/bn_nol_r4.md).
NOL = os.environ.get("MI355X_DP_NOL", "0") == "1"
NOL_USED = [0]  # diagnostics: inner BNs whose output was normalized on load instead of written


def _nol_ok(c, spec) -> bool:
    """can ``spec``'s conv consume the raw tensor ``c`` (shape of its input) with normalize-on-load?"""
    if not NOL:
        return False
    N, C, H, W = c.shape
    K, _, R, S = spec.w.shape
    P, Q = _out_hw(H, R, spec.stride, spec.pad), _out_hw(W, S, spec.stride, spec.pad)
    return bool(_lib.load().mi_conv_nol_ok(N, H, W, C, K, R, S, spec.stride, spec.pad, P, Q))


# ----------------------------------------------------------------------- forward pieces
def _conv_fwd_stats(x, spec, nol=None):
    """conv forward + BN statistics epilogue; ``nol`` = (scale, shift): ``x`` is the raw input of the
    previous BN, normalized (+ ReLU) on load"""
    N, C, H, W = x.shape
    w16 = weight_bf16(spec.w)
    K, _, R, S = spec.w.shape
    P, Q = _out_hw(H, R, spec.stride, spec.pad), _out_hw(W, S, spec.stride, spec.pad)
    lib = _lib.load()
    rows = lib.mi_conv_stat_rows_g(N, H, W, C, K, R, S, spec.stride, spec.pad, P, Q)
    slab = torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, K), dtype=F32, device=x.device)
    y = torch.empty((N, K, P, Q), dtype=BF16, device=x.device, memory_format=CL)
    if nol is not None:
        _lib.call("mi_conv2d_fwd_nol", ptr(x), ptr(w16), ptr(y), ptr(slab), ptr(nol[0]), ptr(nol[1]), N, H, W, C, K,
                  R, S, spec.stride, spec.pad, P, Q, stream_of(x))
        return y, slab, rows
    _lib.call("mi_conv2d_fwd", ptr(x), ptr(w16), ptr(y), ptr(None), ptr(slab), N, H, W, C, K, R, S, spec.stride,
              spec.pad, P, Q, 0, stream_of(x))
    return y, slab, rows


def _bn_fwd(c, slab, rows, bn, relu, res=None, apply=True):
    """BN forward from conv-epilogue statistics.  ``apply=False``: statistics, running-stat update and
    (scale, shift) only -- returns (None, mean, invstd, scale, shift) for a fused consumer."""
    N, C, H, W = c.shape
    dev = c.device
    y = torch.empty_like(c, memory_format=CL) if apply else None
    mean = torch.empty(C, dtype=F32, device=dev)
    invstd = torch.empty(C, dtype=F32, device=dev)
    scale = torch.empty(C, dtype=F32, device=dev)
    shift = torch.empty(C, dtype=F32, device=dev)
    _lib.call("mi_bn_fwd_train", ptr(c), ptr(res), ptr(y), N * H * W, C, bn.eps, bn.momentum, ptr(bn.w), ptr(bn.b),
              ptr(bn.rm), ptr(bn.rv), ptr(bn.nbt), ptr(mean), ptr(invstd), ptr(scale), ptr(shift), ptr(slab),
              int(rows), int(relu), stream_of(c))
    if not apply:
        return None, mean, invstd, scale, shift
    return y, mean, invstd


def _bn_fwd_dual(c, slab, rows, bn, cd, slabd, rowsd, bnd):
    """A block's last BN + ReLU with the projection shortcut's BN folded into the same pass:
    y = relu(bn(c) + bn_d(cd)) -- the shortcut's normalised activation is never materialised.
    Returns (y, mean, invstd, mean_d, invstd_d, bits) -- see _out_apply."""
    _, md, isd, sd, hd = _bn_fwd(cd, slabd, rowsd, bnd, relu=False, apply=False)
    _, m, inv, sc, sh = _bn_fwd(c, slab, rows, bn, relu=True, apply=False)
    y, bits = _out_apply(c, cd, sc, sh, sd, hd)
    return y, m, inv, md, isd, bits


# A block output's ReLU mask as one byte per 8 channels (mi_bn_apply_bits): the next block's conv1
# data-gradient epilogue (epi 5) reads it instead of the bf16 block output -- 1/16 of the bytes in
# the most memory-bound kernels of the backward.  Tensors below this size keep the single-launch
# small-BN path (finalize + apply fused) and the bf16 mask source.
OUT_BITS = os.environ.get("MI355X_DP_OUT_BITS", "1") != "0"
INNER_BITS = os.environ.get("MI355X_DP_INNER_BITS", "1") != "0"  # the same for the inner BNs (bn1 / bn2)
OUT_BITS_MIN = 1 << 22


def _bits_ok(c):
    """emit the mask bytes for BN output ``c``: large enough, and whole bytes per pixel"""
    return OUT_BITS and c.numel() >= OUT_BITS_MIN and c.shape[1] % 8 == 0


def _out_apply(c, res, sc, sh, rsc=None, rsh=None):
    """block output y = relu(c * sc + sh + res') (res' = res, or res * rsc + rsh for a projection
    shortcut's raw conv output) -> (y, bits); bits is None when the mask is not emitted."""
    N, C, H, W = c.shape
    y = torch.empty_like(c, memory_format=CL)
    if _bits_ok(c):
        bits = torch.empty((N, H, W, C // 8), dtype=torch.uint8, device=c.device)
        _lib.call("mi_bn_apply_bits", ptr(c), ptr(res), ptr(y), ptr(bits), N * H * W, C, ptr(sc), ptr(sh), ptr(rsc),
                  ptr(rsh), stream_of(c))
        return y, bits
    if rsc is not None:
        _lib.call("mi_bn_apply_dual", ptr(c), ptr(res), ptr(y), N * H * W, C, ptr(sc), ptr(sh), ptr(rsc), ptr(rsh), 1,
                  stream_of(c))
        return y, None
    return None, None


# ---------------------------------------------------------------------- backward pieces
def _wgrad(x, dy, spec, nol=None):
    """weight gradient into the flat buffer -- on the engine's weight-gradient stream when it has
    one (overlapping this block's data-gradient chain, see functional.WgradStream); ``nol`` =
    (scale, shift): ``x`` is the raw input of the previous BN, normalized (+ ReLU) on load"""
    N, C, H, W = x.shape
    K, _, R, S = spec.w.shape
    P, Q = dy.shape[2], dy.shape[3]
    g = _grad_buffer(spec.w)

    def launch():
        if nol is not None:
            _lib.call("mi_conv2d_wgrad_nol", ptr(x), ptr(dy), ptr(g), ptr(nol[0]), ptr(nol[1]), N, H, W, C, K, R, S,
                      spec.stride, spec.pad, P, Q, stream_of(dy))
            return
        _lib.call("mi_conv2d_wgrad", ptr(x), ptr(dy), ptr(g), N, H, W, C, K, R, S, spec.stride, spec.pad, P, Q,
                  stream_of(dy))
    if _side(spec.w) is not None:
        run_wgrad(spec.w, launch, (x, dy) + (tuple(nol) if nol is not None else ()))
        return None
    launch()
    return _finish_grad(spec.w, g)


def _dgrad(dy, spec, x_shape, out, epi=0, aux=None, aux2=None, mean=None, relu=0, stats=None, flags=0, mbits=None):
    N, C, H, W = x_shape
    K, _, R, S = spec.w.shape
    P, Q = dy.shape[2], dy.shape[3]
    st = stream_of(dy)
    wt = weight_bf16_t(spec.w)
    if mbits is not None:  # ReLU mask bytes instead of the bf16 BN output (epi 4 / 5)
        _lib.call("mi_conv2d_dgrad_ex4", ptr(dy), ptr(wt), ptr(out), N, H, W, C, K, R, S, spec.stride, spec.pad, P,
                  Q, int(epi), ptr(aux), ptr(aux2), ptr(mean), int(relu), ptr(stats), int(flags), ptr(None),
                  ptr(None), ptr(mbits), st)
        return out
    _lib.call("mi_conv2d_dgrad_ex2", ptr(dy), ptr(wt), ptr(out), N, H, W, C, K, R, S, spec.stride, spec.pad, P, Q,
              int(epi), ptr(aux), ptr(aux2), ptr(mean), int(relu), ptr(stats), int(flags), st)
    return out


def _dgrad_bn(dy, spec, y_prev, c_prev, mean_prev, mask=None, bits=None):
    """conv dgrad fused with the relu mask + backward statistics of the BN that produced the conv's
    input: returns (dz, slab, rows).  ``mask`` = that BN's (scale, shift): the mask comes from
    ``c_prev`` (normalize-on-load schedules never write ``y_prev``, which is then None).  ``bits``:
    the mask as bytes of 8 channel bits (_out_apply) instead of reading ``y_prev``."""
    N, C, H, W = c_prev.shape
    lib = _lib.load()
    if isinstance(dy, _Fold):  # the output BN's input gradient folded into this data gradient
        rows = lib.mi_conv_fbb_rows(N * H * W, C, spec.w.shape[0])
        slab = torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, C), dtype=F32, device=dy.dz.device)
        dz = torch.empty_like(c_prev, memory_format=CL)
        _dgrad_fold(dy, spec, c_prev.shape, dz, EPI_BN_BWD, y_prev, c_prev, mean_prev, 1, slab, mbits=bits)
        return dz, slab, rows
    rows = lib.mi_dgrad_stat_rows(N, H, W, C, dy.shape[2], dy.shape[3], spec.stride, spec.w.shape[0],
                                 spec.w.shape[2] * spec.w.shape[3])
    slab = torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, C), dtype=F32, device=dy.device)
    dz = torch.empty_like(c_prev, memory_format=CL)
    if mask is not None:
        K, _, R, S = spec.w.shape
        P, Q = dy.shape[2], dy.shape[3]
        _lib.call("mi_conv2d_dgrad_ex3", ptr(dy), ptr(weight_bf16_t(spec.w)), ptr(dz), N, H, W, C, K, R, S,
                  spec.stride, spec.pad, P, Q, EPI_BN_BWD, ptr(None), ptr(c_prev), ptr(mean_prev), 1, ptr(slab), 0,
                  ptr(mask[0]), ptr(mask[1]), stream_of(dy))
        return dz, slab, rows
    _dgrad(dy, spec, c_prev.shape, dz, EPI_BN_BWD, y_prev, c_prev, mean_prev, 1, slab, mbits=bits)
    return dz, slab, rows


def _bn_bwd(dy, y, c, bn, mean, invstd, relu, dres=None, finish=True):
    """full BN backward (statistics pass included) -> dc, (dgamma, dbeta) for autograd
    (finish=False: the raw gradient buffers, for a later _finish_grad)."""
    N, C, H, W = c.shape
    M = N * H * W
    dev = c.device
    dc = torch.empty_like(c, memory_format=CL)
    gw, gb = _grad_buffer(bn.w), _grad_buffer(bn.b)
    lib = _lib.load()
    part = torch.empty((lib.mi_bn_partial_rows(M, C) + lib.mi_bn_slab_extra_rows(), 2, C), dtype=F32, device=dev)
    coef = torch.empty((3, C), dtype=F32, device=dev)
    _lib.call("mi_bn_bwd_train", ptr(dy), ptr(y), ptr(c), ptr(dc), ptr(dres), M, C, ptr(bn.w), ptr(mean),
              ptr(invstd), ptr(gw), ptr(gb), ptr(coef), ptr(part), int(relu), stream_of(c))
    if not finish:
        return dc, gw, gb
    return dc, _finish_grad(bn.w, gw), _finish_grad(bn.b, gb)


def _bn_bwd_pre(dz, c, bn, mean, invstd, slab, rows):
    """BN backward from dgrad-epilogue statistics (dz already relu-masked)."""
    N, C, H, W = c.shape
    dc = torch.empty_like(c, memory_format=CL)
    gw, gb = _grad_buffer(bn.w), _grad_buffer(bn.b)
    coef = torch.empty((3, C), dtype=F32, device=c.device)
    _lib.call("mi_bn_bwd_train_pre", ptr(dz), ptr(c), ptr(dc), ptr(None), N * H * W, C, ptr(bn.w), ptr(mean),
              ptr(invstd), ptr(gw), ptr(gb), ptr(coef), ptr(slab), int(rows), stream_of(c))
    return dc, _finish_grad(bn.w, gw), _finish_grad(bn.b, gb)


# ------------------------------------------------------------- folded BN backward
# A BatchNorm's input gradient dX = k0 dz + k1 c + k2 (per channel; dz the masked output gradient,
# c the BN input) is consumed by exactly two GEMMs, the data and weight gradients of the conv that
# produced c.  For a 1x1 / stride-1 conv both take it FOLDED instead of reading a materialised dX:
#   dgrad(dX) = [dz | c] x [diag(k0) W | diag(k1) W] + bias(k2 W)   (conv_panel.hip mi_panel_dgrad_fbb)
#   wgrad(dX) = k0 (dz^T x) + k1 (c^T x) + k2 colsum(x)             (gemm_conv.hip mi_conv2d_wgrad_fbb)
# so the BN-backward apply pass (read dz, c; write dX) and both consumers' reads of dX become one
# extra read of c per consumer.  MI355X_DP_BN_FOLD=0 restores the materialised path.
BN_FOLD = os.environ.get("MI355X_DP_BN_FOLD", "1") != "0"
# widest BN (K) folded: 256 (default) keeps the fold to layer 1 (the panel route); 1024 adds the
# layer-3 expansions on the 256-wide kernel (mi_gemm256_dgrad_fbb), which measured slower: ResNet-50
# 13,506 / 13,502 vs 13,654 / 13,679 img/s, ResNet-152 5,585 / 5,564 vs 5,917 / 5,900 -- the 196-tile
# data gradient is MFMA-bound, so doubling its depth costs more than the apply pass it replaces
# (profiles/bn_fold_r6.md)
BN_FOLD_MAXK = int(os.environ.get("MI355X_DP_BN_FOLD_MAXK", "256"))
_FBB_WS = {}  # (weight id, device) -> the folded weight gradient's fp32 workspace (zero between calls)
FOLD_USED = [0]  # diagnostics: BN backwards taken folded


class _Fold:
    """a BN input gradient held unmaterialised: dX = k0 dz + k1 c + k2, coef = (k0, k1, k2) [3][C]"""
    __slots__ = ("dz", "c", "coef")

    def __init__(self, dz, c, coef):
        self.dz, self.c, self.coef = dz, c, coef

    @property
    def shape(self):
        return self.dz.shape


def _fold_ok(spec, x_shape) -> bool:
    """can conv ``spec`` (input shape ``x_shape``) take its output BN's input gradient folded?  Only
    expansions (K > C: the bottleneck conv3s): the folded data gradient reads dz and c (2 K channels)
    where the materialised path wrote and re-read dX, which pays when K is the wide side; for K < C
    the doubled panel depth halves the panel width and the re-reads of [dz | c] per panel cost more
    than the apply pass they replace (tools/bench_fold.py, profiles/bn_fold_r6.md)"""
    if not BN_FOLD:
        return False
    K, C, R, S = spec.w.shape
    # (C <= 256: the folded weight gradient's combine multiplies W by the C x C Gram matrix of x)
    if (R != 1 or S != 1 or spec.stride != 1 or spec.pad != 0 or K % 64 or C % 64 or K <= C or C > 256
            or K > BN_FOLD_MAXK):
        return False
    N, _, H, W = x_shape
    # the panel kernel at the doubled depth, or the 256-wide kernel where the unfolded dgrad runs
    return _lib.load().mi_conv_fbb_route(N * H * W, C, K) > 0


def _bn_bwd_fold(dz, c, bn, mean, invstd, slab, rows):
    """BN backward from dgrad-epilogue statistics, folded: the coefficients only (+ dgamma / dbeta)"""
    N, C, H, W = c.shape
    gw, gb = _grad_buffer(bn.w), _grad_buffer(bn.b)
    coef = torch.empty((3, C), dtype=F32, device=c.device)
    FOLD_USED[0] += 1
    _lib.call("mi_bn_bwd_coef", N * H * W, C, ptr(bn.w), ptr(mean), ptr(invstd), ptr(gw), ptr(gb), ptr(coef),
              ptr(slab), int(rows), stream_of(c))
    return _Fold(dz, c, coef), _finish_grad(bn.w, gw), _finish_grad(bn.b, gb)


def _wgrad_fold(x, fold, spec):
    """_wgrad with the output BN's input gradient folded (mi_conv2d_wgrad_fbb)"""
    N, C, H, W = x.shape
    K, _, R, S = spec.w.shape
    P, Q = fold.dz.shape[2], fold.dz.shape[3]
    g = _grad_buffer(spec.w)
    key = (id(spec.w), x.device.index)
    nf = _lib.load().mi_conv2d_wgrad_fbb_ws_floats(K, C)
    ws = _FBB_WS.get(key)
    if ws is None or ws.numel() < nf:
        ws = _FBB_WS[key] = torch.zeros(nf, dtype=F32, device=x.device)
    w16 = weight_bf16(spec.w)  # [K][1][1][C]: c^T x = W (x^T x)

    def launch():
        _lib.call("mi_conv2d_wgrad_fbb", ptr(x), ptr(fold.dz), ptr(w16), ptr(fold.coef), ptr(g), ptr(ws), N, H, W, C,
                  K, stream_of(fold.dz))
    if _side(spec.w) is not None:
        run_wgrad(spec.w, launch, (x, fold.dz, w16, fold.coef, ws))
        return None
    launch()
    return _finish_grad(spec.w, g)


def _dgrad_fold(fold, spec, x_shape, out, epi=0, aux=None, aux2=None, mean=None, relu=0, stats=None, flags=0,
                mbits=None, acc_src=None):
    """_dgrad with the output BN's input gradient folded (mi_panel_dgrad_fbb); epi 5 accumulates
    ``acc_src`` (default: ``out`` itself) into ``out``"""
    N, C, H, W = x_shape
    K = spec.w.shape[0]
    route = _lib.load().mi_conv_fbb_route(N * H * W, C, K)
    if route == 2:  # the 256-wide kernel: scaled weights [C][2K] and the k2 bias written per call
        assert acc_src is None, "out-of-place accumulate: panel route only"
        wq = torch.empty((C, 2 * K), dtype=BF16, device=fold.dz.device)
        bias = torch.empty(C, dtype=F32, device=fold.dz.device)
        _lib.call("mi_gemm256_dgrad_fbb", ptr(fold.dz), ptr(fold.c), ptr(fold.coef), ptr(weight_bf16_t(spec.w)),
                  ptr(wq), ptr(bias), ptr(out), ptr(stats), int(epi), ptr(aux), ptr(aux2), ptr(mean), int(relu), N, H,
                  W, C, K, (int(flags) >> 1) & 1, ptr(mbits), stream_of(fold.dz))
        return out
    _lib.call("mi_panel_dgrad_fbb", ptr(fold.dz), ptr(fold.c), ptr(fold.coef), ptr(weight_bf16_t(spec.w)), ptr(out),
              N, H, W, C, K, int(epi), ptr(aux), ptr(aux2), ptr(mean), int(relu), ptr(stats), (int(flags) >> 1) & 1,
              ptr(mbits), ptr(acc_src), stream_of(fold.dz))
    return out


def _panel_oop_rows(spec, x_shape) -> int:
    """statistics rows of conv ``spec``'s 1x1 data gradient run on the panel kernel with an
    out-of-place accumulate (mi_panel_dgrad acc_src), 0 if it cannot"""
    K, C, R, S = spec.w.shape
    if R != 1 or S != 1 or spec.stride != 1 or spec.pad != 0 or K % 64:
        return 0
    N, _, H, W = x_shape
    return _lib.load().mi_panel_stat_rows2(N * H * W, C, K, 1)


def _dgrad_panel_oop(dy, spec, x_shape, out, acc_src, epi, aux2=None, mean=None, relu=0, stats=None, flags=0,
                     mbits=None):
    """conv1's accumulating data gradient on the panel kernel, reading the accumulated-into gradient
    from ``acc_src`` and writing ``out`` (epi 3: acc_src rides in aux; epi 5: acc_src)"""
    N, C, H, W = x_shape
    K = spec.w.shape[0]
    aux = acc_src if epi == EPI_ACCUM else None
    _lib.call("mi_panel_dgrad", ptr(dy), ptr(weight_bf16_t(spec.w)), ptr(out), N, H, W, C, K, 1, int(epi), ptr(aux),
              ptr(aux2), ptr(mean), int(relu), ptr(stats), (int(flags) >> 1) & 1, ptr(mbits),
              ptr(acc_src if epi == EPI_ACCUM_BN_BWD else None), stream_of(dy))
    return out


# -------------------------------------------------------------------------- the block
class _ResBlock(torch.autograd.Function):
    """inputs: x, *params (in ``_param_list`` order).  ``specs`` = (convs, bns, has_ds) where the
    main-path convs/bns are [conv1, conv2(, conv3)] / [bn1, bn2(, bn3)] and the downsample pair,
    if any, is appended last."""

    @staticmethod
    def forward(ctx, x, specs, prev_bnsrc, *params):
        ctx.params_order = params
        convs, bns, has_ds = specs
        n_main = len(convs) - (1 if has_ds else 0)
        x = _nhwc(x)
        saved_c, saved_y, saved_m, saved_i = [], [], [], []
        out_bits = None          # the block output's ReLU mask bytes (_out_apply), for the next block
        inner_bits = [None] * n_main  # inner BNs' ReLU mask bytes, for the data gradients
        aux = _aux_stream(x.device) if has_ds else None
        if aux is not None:
            # shortcut conv + its BN statistics / finalize, concurrently with the main chain
            main = torch.cuda.current_stream(x.device)
            aux.wait_stream(main)
            with torch.cuda.stream(aux):
                cd, slabd, rowsd = _conv_fwd_stats(x, convs[-1])
                _, md, isd, sd, hd = _bn_fwd(cd, slabd, rowsd, bns[-1], relu=False, apply=False)
        h = x
        nol = None               # (scale, shift) when h is a raw BN input normalized on load
        saved_nol = []
        for i in range(n_main):
            c, slab, rows = _conv_fwd_stats(h, convs[i], nol)
            last = i == n_main - 1
            if last:
                if has_ds and aux is not None:
                    _, m, inv, sc, sh = _bn_fwd(c, slab, rows, bns[i], relu=True, apply=False)
                    main.wait_stream(aux)
                    y, out_bits = _out_apply(c, cd, sc, sh, sd, hd)
                elif has_ds:
                    cd, slabd, rowsd = _conv_fwd_stats(x, convs[-1])
                    y, m, inv, md, isd, out_bits = _bn_fwd_dual(c, slab, rows, bns[i], cd, slabd, rowsd, bns[-1])
                elif _bits_ok(c):
                    _, m, inv, sc, sh = _bn_fwd(c, slab, rows, bns[i], relu=True, apply=False)
                    y, out_bits = _out_apply(c, x, sc, sh)
                else:
                    y, m, inv = _bn_fwd(c, slab, rows, bns[i], relu=True, res=x)
            elif _nol_ok(c, convs[i + 1]):
                # inner BN, consumer normalizes on load: statistics / running stats / (scale, shift)
                # only -- y is never materialised
                _, m, inv, sc, sh = _bn_fwd(c, slab, rows, bns[i], relu=True, apply=False)
                y = None
                nol = (sc, sh)
                NOL_USED[0] += 1
            else:
                if INNER_BITS and _bits_ok(c):
                    # inner BN: y for the next conv (forward, weight gradient) plus its ReLU mask bytes
                    # for that conv's data-gradient epilogue
                    _, m, inv, sc, sh = _bn_fwd(c, slab, rows, bns[i], relu=True, apply=False)
                    y, inner_bits[i] = _out_apply(c, None, sc, sh)
                else:
                    y, m, inv = _bn_fwd(c, slab, rows, bns[i], relu=True)
                nol = None
            saved_c.append(c); saved_y.append(y); saved_m.append(m); saved_i.append(inv)
            saved_nol.append(nol if y is None else None)
            h = y if y is not None else c
        # y of a normalize-on-load BN is None: its (scale, shift) ride in the y slot's place
        ys_t = [y if y is not None else saved_nol[k][0] for k, y in enumerate(saved_y)]
        nol_t = [saved_nol[k][1] if saved_nol[k] is not None else saved_c[k] for k in range(n_main)]
        ctx.nol_flags = [s_ is not None for s_ in saved_nol]
        tensors = [x] + saved_c + ys_t + saved_m + saved_i + nol_t
        if has_ds:
            tensors += [cd, md, isd]
        ctx.save_for_backward(*tensors)
        ctx.specs = specs
        ctx.n_main = n_main
        # read by the next block (input = this output): its last BN's input, mean and ReLU mask bytes
        ctx.out_bnsrc = (saved_c[-1], saved_m[-1], out_bits)
        ctx.inner_bits = inner_bits
        ctx.prev_bnsrc = prev_bnsrc
        return h

    @staticmethod
    def _shortcut_backward(x, dyd, dx, cd, md, isd, convs, bns, grads):
        """projection shortcut backward on the current stream: its BN backward (affine gradients
        returned raw), weight gradient, and data gradient written into dx -> (acc_flags, (gw, gb))"""
        ds = convs[-1]
        if _fold_ok(ds, x.shape):
            # a stride-1 expansion (layer 1's 64 -> 256): statistics + coefficients, then the BN's
            # input gradient folded into the shortcut conv's data and weight gradients (see _Fold)
            N, C, H, W = cd.shape
            M = N * H * W
            lib = _lib.load()
            gw, gb = _grad_buffer(bns[-1].w), _grad_buffer(bns[-1].b)
            coef = torch.empty((3, C), dtype=F32, device=cd.device)
            part = torch.empty((lib.mi_bn_partial_rows(M, C) + lib.mi_bn_slab_extra_rows(), 2, C), dtype=F32,
                               device=cd.device)
            FOLD_USED[0] += 1
            _lib.call("mi_bn_bwd_train", ptr(dyd), ptr(dyd), ptr(cd), ptr(None), ptr(None), M, C, ptr(bns[-1].w),
                      ptr(md), ptr(isd), ptr(gw), ptr(gb), ptr(coef), ptr(part), 0, stream_of(cd))
            fold = _Fold(dyd, cd, coef)
            grads[id(ds.w)] = _wgrad_fold(x, fold, ds)
            _dgrad_fold(fold, ds, x.shape, dx)                      # dx = dgrad_ds
            return 0, (gw, gb)
        dcd, gw, gb = _bn_bwd(dyd, dyd, cd, bns[-1], md, isd, relu=0, finish=False)
        grads[id(convs[-1].w)] = _wgrad(x, dcd, convs[-1])
        if ds.stride == 2 and ds.pad == 0 and ds.w.shape[2] == 1 and ds.w.shape[3] == 1:
            # 1x1 / stride-2 shortcut: its data gradient lives on the even pixels only -- write
            # just those and let conv1's dgrad read the sum there (DGRAD_SPARSE / DGRAD_ACC_EVEN)
            _dgrad(dcd, ds, x.shape, dx, flags=DGRAD_SPARSE)
            return DGRAD_ACC_EVEN, (gw, gb)
        _dgrad(dcd, ds, x.shape, dx)                               # dx = dgrad_ds
        return 0, (gw, gb)

    @staticmethod
    def backward(ctx, dout):
        convs, bns, has_ds = ctx.specs
        n = ctx.n_main
        t = ctx.saved_tensors
        x = t[0]
        cs, ys, ms, invs = t[1:1 + n], list(t[1 + n:1 + 2 * n]), t[1 + 2 * n:1 + 3 * n], t[1 + 3 * n:1 + 4 * n]
        shs = t[1 + 4 * n:1 + 5 * n]
        nols = [(ys[k], shs[k]) if ctx.nol_flags[k] else None for k in range(n)]
        ys = [None if ctx.nol_flags[k] else ys[k] for k in range(n)]
        if has_ds:
            cd, md, isd = t[1 + 5 * n:]
        dout = _nhwc(dout)
        grads = {}
        hand = _HANDOFF.pop((dout.data_ptr(), dout.device.index), None)
        if hand is not None and not (hand[2] == dout._version and hand[3] == cs[-1].data_ptr()
                                     and dout.is_contiguous(memory_format=CL)):
            hand = None
        # folded BN backward (see _Fold): conv i takes bn i's input gradient folded when it is a
        # 1x1 / stride-1 conv the panel kernel runs at the doubled depth (never with normalize-on-load)
        in_shapes = [x.shape] + [c.shape for c in cs[:-1]]
        fold = [not any(ctx.nol_flags) and _fold_ok(convs[i], in_shapes[i]) for i in range(n)]
        acc_src = None  # conv1's epi-5 accumulate source when dx may not alias dout
        if hand is not None:
            HANDOFF_USED[0] += 1
            # dout is already dz3 (masked) with bn3's statistics computed by the next block: it IS
            # the residual-path gradient, so it doubles as dyd / the initial dx (no copy)
            if fold[n - 1] and (has_ds or fold[0] or _panel_oop_rows(convs[0], x.shape) > 0):
                # folded: conv3's weight gradient reads dout on the side stream, so with an identity
                # shortcut conv1's data gradient must not accumulate into dout in place -- it reads
                # dout (acc_src) and writes a fresh dx (on the panel kernel, folded or not)
                dc, gw, gb = _bn_bwd_fold(dout, cs[-1], bns[n - 1], ms[-1], invs[-1], hand[0], hand[1])
                if not has_ds:
                    acc_src = dout
            else:
                dc, gw, gb = _bn_bwd_pre(dout, cs[-1], bns[n - 1], ms[-1], invs[-1], hand[0], hand[1])
            dyd = dout if has_ds else None
            dx = torch.empty_like(x, memory_format=CL) if (has_ds or acc_src is not None) else dout
        else:
            dx = torch.empty_like(x, memory_format=CL)
            # last BN: relu + residual; dres -> dx (identity) or the downsample BN's output gradient
            dyd = torch.empty_like(ys[-1], memory_format=CL) if has_ds else None
            dc, gw, gb = _bn_bwd(dout, ys[-1], cs[-1], bns[n - 1], ms[-1], invs[-1], relu=1,
                                 dres=dyd if has_ds else dx)
        grads[id(bns[n - 1].w)], grads[id(bns[n - 1].b)] = gw, gb
        acc_flags = 0
        aux = _aux_stream(x.device) if has_ds else None
        if aux is not None:
            # shortcut branch (BN backward, weight gradient, data gradient into dx) concurrently with
            # the main chain; its BN affine gradients are signalled after the join below
            main = torch.cuda.current_stream(x.device)
            aux.wait_stream(main)
            with torch.cuda.stream(aux):
                acc_flags, dsd = _ResBlock._shortcut_backward(x, dyd, dx, cd, md, isd, convs, bns, grads)
        for i in range(n - 1, 0, -1):
            nol = nols[i - 1]
            inp = ys[i - 1] if nol is None else cs[i - 1]
            if isinstance(dc, _Fold):
                grads[id(convs[i].w)] = _wgrad_fold(inp, dc, convs[i])
            else:
                grads[id(convs[i].w)] = _wgrad(inp, dc, convs[i], nol)
            dz, slab, rows = _dgrad_bn(dc, convs[i], ys[i - 1], cs[i - 1], ms[i - 1], mask=nol,
                                       bits=ctx.inner_bits[i - 1])
            if fold[i - 1]:
                dc, gw, gb = _bn_bwd_fold(dz, cs[i - 1], bns[i - 1], ms[i - 1], invs[i - 1], slab, rows)
            else:
                dc, gw, gb = _bn_bwd_pre(dz, cs[i - 1], bns[i - 1], ms[i - 1], invs[i - 1], slab, rows)
            grads[id(bns[i - 1].w)], grads[id(bns[i - 1].b)] = gw, gb
        if isinstance(dc, _Fold):
            grads[id(convs[0].w)] = _wgrad_fold(x, dc, convs[0])
        else:
            grads[id(convs[0].w)] = _wgrad(x, dc, convs[0])
        if aux is not None:
            main.wait_stream(aux)  # conv1's dgrad accumulates into the shortcut's dx
            gw, gb = dsd
            grads[id(bns[-1].w)], grads[id(bns[-1].b)] = _finish_grad(bns[-1].w, gw), _finish_grad(bns[-1].b, gb)
        elif has_ds:
            acc_flags, (gw, gb) = _ResBlock._shortcut_backward(x, dyd, dx, cd, md, isd, convs, bns, grads)
            grads[id(bns[-1].w)], grads[id(bns[-1].b)] = _finish_grad(bns[-1].w, gw), _finish_grad(bns[-1].b, gb)
        if ctx.prev_bnsrc is not None:
            # dx = mask_prev * (dx + dgrad_1) + the previous block's last-BN backward statistics
            c_prev, m_prev, bits_prev = ctx.prev_bnsrc
            N, C, H, W = x.shape
            lib = _lib.load()
            rows = lib.mi_dgrad_stat_rows(N, H, W, C, dc.shape[2], dc.shape[3], convs[0].stride,
                                          convs[0].w.shape[0], convs[0].w.shape[2] * convs[0].w.shape[3])
            if isinstance(dc, _Fold):
                rows = lib.mi_conv_fbb_rows(N * H * W, C, convs[0].w.shape[0])
            elif acc_src is not None:
                rows = _panel_oop_rows(convs[0], x.shape)
            slab = torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, C), dtype=F32, device=dx.device)
            if isinstance(dc, _Fold):
                _dgrad_fold(dc, convs[0], x.shape, dx, EPI_ACCUM_BN_BWD, x, c_prev, m_prev, 1, slab, flags=acc_flags,
                            mbits=bits_prev, acc_src=acc_src)
            elif acc_src is not None:
                _dgrad_panel_oop(dc, convs[0], x.shape, dx, acc_src, EPI_ACCUM_BN_BWD, c_prev, m_prev, 1, slab,
                                 flags=acc_flags, mbits=bits_prev)
            else:
                _dgrad(dc, convs[0], x.shape, dx, EPI_ACCUM_BN_BWD, x, c_prev, m_prev, 1, slab, flags=acc_flags,
                       mbits=bits_prev)
            _HANDOFF[(dx.data_ptr(), dx.device.index)] = (slab, rows, dx._version, c_prev.data_ptr())
        elif isinstance(dc, _Fold):
            # dx += dgrad_1 (epi 3 reads the accumulated-into gradient from aux)
            _dgrad_fold(dc, convs[0], x.shape, dx, EPI_ACCUM, acc_src if acc_src is not None else dx, flags=acc_flags)
        elif acc_src is not None:
            _dgrad_panel_oop(dc, convs[0], x.shape, dx, acc_src, EPI_ACCUM, flags=acc_flags)
        else:
            _dgrad(dc, convs[0], x.shape, dx, EPI_ACCUM, dx, flags=acc_flags)   # dx += dgrad_1
        ctx.prev_bnsrc = None
        ctx.out_bnsrc = None
        ctx.inner_bits = None
        out = [dx, None, None]
        for p in ctx.params_order:
            out.append(grads.get(id(p)))
        return tuple(out)


def _specs(block):
    convs = [block.conv1, block.conv2] + ([block.conv3] if hasattr(block, "conv3") else [])
    bns = [block.bn1, block.bn2] + ([block.bn3] if hasattr(block, "bn3") else [])
    has_ds = block.downsample is not None
    if has_ds:
        convs.append(block.downsample[0])
        bns.append(block.downsample[1])
    return convs, bns, has_ds


def fusable(block, x) -> bool:
    """The fused node covers the native training path: CUDA, grad enabled, BN in training mode
    with running statistics and a fixed momentum, every conv a native MFMA conv (C % 64 == 0)."""
    from mi355x_dp.models.layers import BatchNorm2d, Conv2d
    if not (x.is_cuda and x.dtype == torch.bfloat16 and torch.is_grad_enabled() and block.training):
        return False
    convs, bns, _ = _specs(block)
    for c in convs:
        if not isinstance(c, Conv2d) or c.bias is not None or c.groups != 1 or c.in_channels % 64 != 0 \
                or c.out_channels % 64 != 0 or c.stride[0] > 2 or c.dilation[0] != 1 or c.stride[0] != c.stride[1]:
            return False
    for b in bns:
        if not isinstance(b, BatchNorm2d) or not b.track_running_stats or not b.affine or b.momentum is None:
            return False
    return True


def res_block(block, x):
    """Run a BasicBlock / Bottleneck as one fused autograd node (caller checked ``fusable``)."""
    convs, bns, has_ds = _specs(block)
    cspecs = tuple(_ConvSpec(c) for c in convs)
    bspecs = tuple(_BNSpec(b) for b in bns)
    params = [c.w for c in cspecs]
    for b in bspecs:
        params += [b.w, b.b]
    prev = x.grad_fn
    prev_bnsrc = getattr(prev, "out_bnsrc", None) if type(prev).__name__ == "_ResBlockBackward" else None
    if prev_bnsrc is None:
        _HANDOFF.clear()  # first block of a forward: drop hand-offs a skipped backward left behind
    return _ResBlock.apply(x, (cspecs, bspecs, has_ds), prev_bnsrc, *params)
