"""Numerics of the persistent resident-weight 1x1 conv kernel (csrc/kernels/conv_panel.hip) against a
plain PyTorch fp32 reference of the same conv (inputs rounded to bf16 first) and against the 128-tile
nt_kernel it replaces: the MFMA chain per output element is the same instruction sequence, so the
bf16 output must match bit for bit; the BatchNorm statistics slab (one row per block) must sum to the
statistics of the rounded output.  Shapes: every panel width / ring depth the dispatcher picks for
ResNet-50, the 1x1 stride-2 gather, and row counts that are not a multiple of the
32-row wave unit."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last
BF = torch.bfloat16

# (N, C, H, K, stride): panel 256/128/64 wide, ring depth 4/3, gather, ragged M
SHAPES = [
    (4, 64, 56, 256, 1),    # layer-1 expansion: BN 256, K 64
    (4, 256, 56, 64, 1),    # layer-1 reduction: BN 64, K 256
    (4, 64, 56, 64, 1),     # layer-1 first conv: BN 64, K 64
    (2, 256, 56, 128, 1),   # layer-2 first conv: BN 128, 64 KB panel (3 slots)
    (4, 128, 28, 512, 1),   # layer-2 expansion: BN 256 x 2 panels
    (4, 256, 56, 512, 2),   # layer-2 downsample: stride-2 gather, 4 panels
    (3, 256, 14, 1024, 1),  # layer-3 expansion, M = 588 (ragged units), 8 panels
    (2, 512, 28, 128, 1),   # K 512: BN 64 panels
    (1, 64, 7, 64, 1),      # tiny: fewer units than wave slots
    (3, 1024, 14, 256, 1),  # K 1024: 32-column panels (64 KB, 3 slots), 8 panels
    (2, 1024, 9, 96, 1),    # K 1024, N 96: 32-column panels, ragged M
    (4, 64, 56, 64, 1, 3),  # layer-1 3x3 (72 KB panel, 2 slots, nine gathered taps)
    (3, 64, 13, 64, 1, 3),  # 3x3, odd spatial size, ragged M
]


@pytest.fixture(scope="module")
def lib():
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    lib = _lib.load(True)  # fail loudly if the extension is missing
    yield lib
    lib.mi_set_panel(1)


def rel_err(a, b):
    a = a.detach().float()
    b = b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


def _fwd(lib, x, w, stride, stats):
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    N, C, H, _ = x.shape
    K, R = w.shape[0], w.shape[2]
    pad = R // 2
    P = (H + 2 * pad - R) // stride + 1
    y = torch.empty(N, K, P, P, dtype=BF, device="cuda", memory_format=CL)
    _lib.call("mi_conv2d_fwd", ptr(x), ptr(w), ptr(y), ptr(None), ptr(stats), N, H, H, C, K, R, R, stride, pad, P, P,
              0, stream_of(x))
    return y


@pytest.mark.parametrize("shape", SHAPES)
def test_panel_conv1x1_fwd(lib, shape):
    torch.manual_seed(1)
    N, C, H, K, s = shape[:5]
    R = shape[5] if len(shape) > 5 else 1
    pad = R // 2
    P = (H + 2 * pad - R) // s + 1
    M = N * P * P
    x = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.1).to(BF).contiguous(memory_format=CL)
    lib.mi_set_panel(6)  # any row count, 3x3 included
    rows = lib.mi_panel_stat_rows(M, K, C * R * R)
    assert rows > 0, "shape not routed to the panel kernel"
    assert lib.mi_conv_stat_rows_g(N, H, H, C, K, R, R, s, pad, P, P) == rows
    slab = torch.full((rows + 8, 2, K), float("nan"), device="cuda")
    y = _fwd(lib, x, w, s, slab)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float(), w.float(), None, s, pad)
    assert rel_err(y, ref) < 1e-2
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, K)
    assert torch.isfinite(slab[:rows]).all(), "statistics rows left unwritten"
    assert rel_err(slab[:rows, 0].sum(0), yf.sum(0)) < 1e-3
    assert rel_err(slab[:rows, 1].sum(0), (yf * yf).sum(0)) < 1e-3
    # the replaced 128-tile kernel: same MFMA sequence per element -> identical bf16 output
    lib.mi_set_panel(0)
    lib.mi_set_nt_split_blocks(0)  # the unsplit k-order
    rows0 = lib.mi_conv_stat_rows_g(N, H, H, C, K, R, R, s, pad, P, P)
    y0 = _fwd(lib, x, w, s, torch.empty(rows0, 2, K, device="cuda"))
    lib.mi_set_nt_split_blocks(128)
    lib.mi_set_panel(6)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    # no statistics requested: the plain store path
    y2 = _fwd(lib, x, w, s, None)
    torch.cuda.synchronize()
    assert torch.equal(y2, y)


# data gradient (dx channels C, dy channels K): panel widths 256 / 64 (4 and 1 waves across), 64 KB
# panels (3 slots), 2 panels, ragged M
DGRAD_SHAPES = [
    (4, 56, 256, 64), (4, 56, 64, 256), (2, 56, 256, 128), (4, 28, 512, 128), (4, 28, 128, 512), (3, 14, 1024, 256),
    (3, 14, 256, 1024),  # K 1024: 32-column panels
    (4, 56, 64, 64, 3), (3, 13, 64, 64, 3),  # 3x3 / pad 1: the flipped taps of wt = [C][3][3][K]
]
# (epi, mask: "bits" | "y" | None, stats, flags): flags bit 1 = the accumulated-into gradient exists
# only at even (h, w) (a stride-2 downsample's sparse data gradient)
DGRAD_EPIS = [(0, None, False, 0), (3, None, False, 0), (4, "bits", True, 0), (5, "bits", True, 0),
              (5, "bits", True, 2), (4, "y", True, 0), (3, None, False, 2)]


def _dgrad(lib, dy, wt, dx, epi, aux, x, mean, mask, bits, stats, flags):
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    N, K, H, W = dy.shape
    C, R = dx.shape[1], wt.shape[1]
    _lib.call("mi_conv2d_dgrad_ex4", ptr(dy), ptr(wt), ptr(dx), N, H, W, C, K, R, R, 1, R // 2, H, W, epi,
              ptr(aux), ptr(x), ptr(mean), 1 if mask else 0, ptr(stats), flags, ptr(None), ptr(None),
              ptr(bits if mask == "bits" else None), stream_of(dy))


@pytest.mark.parametrize("epi,mask,stats,flags", DGRAD_EPIS)
@pytest.mark.parametrize("shape", DGRAD_SHAPES)
def test_panel_dgrad1x1(lib, shape, epi, mask, stats, flags):
    """the 1x1 data gradient with nt_kernel's fused epilogues (residual add, BN backward with the ReLU
    mask from mask bytes or from the BN output, the (sum dz, sum dz (x - mean)) statistics, the
    sparse even-pixel accumulate): bf16 output bit for bit equal to the 128-tile kernel's, statistics
    equal up to fp32 summation order"""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    torch.manual_seed(2)
    N, H, C, K = shape[:4]
    R = shape[4] if len(shape) > 4 else 1
    if R == 3 and flags:
        pytest.skip("the sparse even-pixel accumulate only follows 1x1 downsample data gradients")
    M = N * H * H
    dy = torch.randn(N, K, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.1).to(BF).contiguous(memory_format=CL)
    wt = torch.empty(C, R, R, K, dtype=BF, device="cuda")
    _lib.call("mi_conv_wtrans", ptr(w), ptr(wt), K, R * R, C, stream_of(dy))
    base = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
    if flags & 2:  # only even (h, w) defined: odd pixels hold garbage the kernel must not read
        base[:, :, 1::2, :] = float("nan")
        base[:, :, :, 1::2] = float("nan")
    x = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
    y = torch.relu(torch.randn(N, C, H, H, device="cuda")).to(BF).contiguous(memory_format=CL)
    aux = base if epi == 3 else (y if mask == "y" else None)  # the residual, or the BN output for the mask
    yb = (y.permute(0, 2, 3, 1).reshape(M, C // 8, 8) > 0).to(torch.int32)
    bits = (yb << torch.arange(8, device="cuda", dtype=torch.int32)).sum(-1).to(torch.uint8).contiguous()
    mean = torch.randn(C, device="cuda") * 0.1
    out = {}
    for mode in (6, 0):
        lib.mi_set_panel(mode)
        lib.mi_set_nt_split_blocks(0)
        rows = lib.mi_dgrad_stat_rows(N, H, H, C, H, H, 1, K, R * R)
        if mode == 6:
            assert rows == lib.mi_panel_stat_rows2(M, C, R * R * K, 1) > 0, "not routed to the panel kernel"
        sl = torch.full((rows + 8, 2, C), float("nan"), device="cuda") if stats else None
        dx = base.clone() if epi == 5 else torch.empty_like(base)
        _dgrad(lib, dy, wt, dx, epi, aux, x, mean, mask, bits, sl, flags)
        torch.cuda.synchronize()
        out[mode] = (dx, sl[:rows] if stats else None)
    lib.mi_set_nt_split_blocks(128)
    lib.mi_set_panel(6)
    dx_p, sl_p = out[6]
    dx_o, sl_o = out[0]
    if epi == 3 and flags & 2:
        # epi 3 reads its residual at every pixel; the NaN-poisoned odd ones propagate alike
        assert torch.equal(dx_p.isnan(), dx_o.isnan())
        dx_p, dx_o = torch.nan_to_num(dx_p), torch.nan_to_num(dx_o)
    assert torch.equal(dx_p, dx_o)
    if epi == 0:
        ref = torch.nn.grad.conv2d_input(dx_p.shape, w.float(), dy.float(), 1, R // 2)
        assert rel_err(dx_p, ref) < 1e-2
    if stats:
        assert torch.isfinite(sl_p).all(), "statistics rows left unwritten"
        for k in (0, 1):
            assert rel_err(sl_p[:, k].sum(0), sl_o[:, k].sum(0)) < 1e-4


# folded BN backward: (N, H, C = dx channels, K = dz / c channels)
FBB_SHAPES = [(4, 56, 64, 256), (4, 56, 256, 64), (4, 28, 512, 128), (3, 14, 1024, 256), (2, 13, 64, 64)]


def _fbb_inputs(N, H, C, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    dz = torch.randn(N, K, H, H, device="cuda", generator=g).to(BF).contiguous(memory_format=CL)
    c = (torch.randn(N, K, H, H, device="cuda", generator=g) * 2 + 0.3).to(BF).contiguous(memory_format=CL)
    coef = torch.stack([torch.rand(K, device="cuda", generator=g) + 0.5,
                        torch.randn(K, device="cuda", generator=g) * 0.1,
                        torch.randn(K, device="cuda", generator=g) * 0.1]).contiguous()
    w = (torch.randn(K, C, 1, 1, device="cuda", generator=g) * (1.0 / K) ** 0.5).to(BF).contiguous(memory_format=CL)
    dX = dz.float() * coef[0].view(1, K, 1, 1) + c.float() * coef[1].view(1, K, 1, 1) + coef[2].view(1, K, 1, 1)
    return dz, c, coef, w, dX


@pytest.mark.parametrize("epi", [0, 4, 5])
@pytest.mark.parametrize("shape", FBB_SHAPES)
def test_panel_dgrad_fbb(lib, shape, epi):
    """the 1x1 data gradient of a BN's input gradient folded into the GEMM ([dz | c] against
    [diag(k0) W | diag(k1) W] plus the k2 bias) against fp32 math on the materialised dX, with the
    BN-backward epilogue of the conv's own input BN (mask bytes + statistics) and the residual
    accumulate (epi 5, in place and out of place)"""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    N, H, C, K = shape
    M = N * H * H
    dz, c, coef, w, dX = _fbb_inputs(N, H, C, K, 7)
    wt = torch.empty(C, 1, 1, K, dtype=BF, device="cuda")
    st = stream_of(dz)
    _lib.call("mi_conv_wtrans", ptr(w), ptr(wt), K, 1, C, st)
    lib.mi_set_panel(6)
    try:
        rows = lib.mi_panel_fbb_rows(M, C, K)
        if rows <= 0:
            pytest.skip("not eligible for the folded path (panel depth)")
        ref = torch.nn.grad.conv2d_input((N, C, H, H), w.float(), dX, 1, 0)  # fp32 dgrad of the materialised dX
        base = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        yb = torch.relu(torch.randn(N, C, H, H, device="cuda")).to(BF).contiguous(memory_format=CL)
        ybits = (yb.permute(0, 2, 3, 1).reshape(M, C // 8, 8) > 0).to(torch.int32)
        bits = (ybits << torch.arange(8, device="cuda", dtype=torch.int32)).sum(-1).to(torch.uint8).contiguous()
        xin = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        mean = torch.randn(C, device="cuda") * 0.1
        mask = (yb > 0).float()
        outs = []
        for oop in ((False, True) if epi == 5 else (False,)):
            dx = base.clone() if (epi == 5 and not oop) else torch.empty_like(base)
            sl = torch.full((rows + 8, 2, C), float("nan"), device="cuda") if epi >= 4 else None
            _lib.call("mi_panel_dgrad_fbb", ptr(dz), ptr(c), ptr(coef), ptr(wt), ptr(dx), N, H, H, C, K, epi, ptr(None),
                      ptr(xin), ptr(mean), 1, ptr(sl), 0, ptr(bits if epi >= 4 else None), ptr(base if oop else None),
                      st)
            torch.cuda.synchronize()
            outs.append(dx)
            if epi == 0:
                want = ref
            elif epi == 4:
                want = ref.to(BF).float() * mask
            else:
                want = (ref.to(BF).float() + base.float()) * mask
            assert rel_err(dx, want) < 2e-2, (oop, rel_err(dx, want))
            if epi >= 4:
                assert torch.isfinite(sl[:rows]).all()
                wf = want.permute(0, 2, 3, 1).reshape(M, C)
                xf = xin.float().permute(0, 2, 3, 1).reshape(M, C)
                assert rel_err(sl[:rows, 0].sum(0), wf.sum(0)) < 3e-2
                assert rel_err(sl[:rows, 1].sum(0), (wf * (xf - mean)).sum(0)) < 3e-2
        if len(outs) == 2:
            assert torch.equal(outs[0], outs[1])  # out of place == in place
    finally:
        lib.mi_set_panel(1)


@pytest.mark.parametrize("shape", FBB_SHAPES)
def test_wgrad_fbb(lib, shape):
    """the weight gradient of a 1x1 conv against its output BN's input gradient, folded:
    k0 (dz^T x) + k1 W (x^T x) + k2 colsum(x) (c = x W^T, so c^T x = W G) from ONE TN GEMM over
    [dz | x] with the input's column sums per split, against fp32 math on the materialised dX from the
    stored bf16 c; accumulates into dW; leaves its workspace zeroed for the next call"""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    N, H, C, K = shape
    dz, _, coef, w, _ = _fbb_inputs(N, H, C, K, 9)
    x = torch.relu(torch.randn(N, C, H, H, device="cuda")).to(BF).contiguous(memory_format=CL)
    c = F.conv2d(x.float(), w.float()).to(BF)  # the forward conv's stored output
    dX = dz.float() * coef[0].view(1, K, 1, 1) + c.float() * coef[1].view(1, K, 1, 1) + coef[2].view(1, K, 1, 1)
    ref = torch.nn.grad.conv2d_weight(x.float(), (K, C, 1, 1), dX, 1, 0).permute(0, 2, 3, 1).contiguous()
    ws = torch.zeros(lib.mi_conv2d_wgrad_fbb_ws_floats(K, C), device="cuda")
    dw0 = torch.randn(K, 1, 1, C, device="cuda")
    dw = dw0.clone()
    st = stream_of(dz)
    for rep in range(2):
        _lib.call("mi_conv2d_wgrad_fbb", ptr(x), ptr(dz), ptr(w), ptr(coef), ptr(dw), ptr(ws), N, H, H, C, K, st)
        torch.cuda.synchronize()
        assert rel_err(dw - dw0, ref * (rep + 1)) < 1e-2, (rep, rel_err(dw - dw0, ref * (rep + 1)))
        assert float(ws[:(K + C) * C].abs().max()) == 0.0  # T and G re-zeroed


@pytest.mark.parametrize("epi", [0, 4])
@pytest.mark.parametrize("shape", [(4, 14, 256, 1024), (3, 13, 256, 512)])
def test_gemm256_dgrad_fbb(lib, shape, epi):
    """the folded data gradient on the 256-wide kernel (convs too deep for the panel at 2K): [dz | c]
    gathered from two tensors by k-tile against the scaled weights written per call, the k2 bias in
    the epilogue, against fp32 math on the materialised dX (forced onto the 256-wide kernel)"""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    N, H, C, K = shape
    M = N * H * H
    dz, c, coef, w, dX = _fbb_inputs(N, H, C, K, 13)
    wt = torch.empty(C, 1, 1, K, dtype=BF, device="cuda")
    st = stream_of(dz)
    _lib.call("mi_conv_wtrans", ptr(w), ptr(wt), K, 1, C, st)
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.float(), dX, 1, 0)
    yb = torch.relu(torch.randn(N, C, H, H, device="cuda")).to(BF).contiguous(memory_format=CL)
    ybits = (yb.permute(0, 2, 3, 1).reshape(M, C // 8, 8) > 0).to(torch.int32)
    bits = (ybits << torch.arange(8, device="cuda", dtype=torch.int32)).sum(-1).to(torch.uint8).contiguous()
    xin = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
    mean = torch.randn(C, device="cuda") * 0.1
    rows = lib.mi_g256_stat_rows(M, C, 2 * K)
    sl = torch.full((rows + 8, 2, C), float("nan"), device="cuda") if epi == 4 else None
    wq = torch.empty(C, 2 * K, dtype=BF, device="cuda")
    bias = torch.empty(C, device="cuda")
    dx = torch.empty(N, C, H, H, dtype=BF, device="cuda", memory_format=CL)
    _lib.call("mi_gemm256_dgrad_fbb", ptr(dz), ptr(c), ptr(coef), ptr(wt), ptr(wq), ptr(bias), ptr(dx), ptr(sl), epi,
              ptr(None), ptr(xin), ptr(mean), 1, N, H, H, C, K, 0, ptr(bits if epi == 4 else None), st)
    torch.cuda.synchronize()
    want = ref if epi == 0 else ref.to(BF).float() * (yb > 0).float()
    assert rel_err(dx, want) < 2e-2, rel_err(dx, want)
    assert rel_err(bias, (coef[2].view(1, K) * wt.view(C, K).float()).sum(1)) < 1e-4
    if epi == 4:
        assert torch.isfinite(sl[:rows]).all()
        wf = want.permute(0, 2, 3, 1).reshape(M, C)
        xf = xin.float().permute(0, 2, 3, 1).reshape(M, C)
        assert rel_err(sl[:rows, 0].sum(0), wf.sum(0)) < 3e-2
        assert rel_err(sl[:rows, 1].sum(0), (wf * (xf - mean)).sum(0)) < 3e-2
