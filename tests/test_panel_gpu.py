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
    K = w.shape[0]
    P = (H - 1) // stride + 1
    y = torch.empty(N, K, P, P, dtype=BF, device="cuda", memory_format=CL)
    _lib.call("mi_conv2d_fwd", ptr(x), ptr(w), ptr(y), ptr(None), ptr(stats), N, H, H, C, K, 1, 1, stride, 0, P, P, 0,
              stream_of(x))
    return y


@pytest.mark.parametrize("shape", SHAPES)
def test_panel_conv1x1_fwd(lib, shape):
    torch.manual_seed(1)
    N, C, H, K, s = shape
    P = (H - 1) // s + 1
    M = N * P * P
    x = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
    w = (torch.randn(K, C, 1, 1, device="cuda") * 0.1).to(BF).contiguous(memory_format=CL)
    lib.mi_set_panel(2)  # any row count
    rows = lib.mi_panel_stat_rows(M, K, C)
    assert rows > 0, "shape not routed to the panel kernel"
    assert lib.mi_conv_stat_rows_g(N, H, H, C, K, 1, 1, s, 0, P, P) == rows
    slab = torch.full((rows + 8, 2, K), float("nan"), device="cuda")
    y = _fwd(lib, x, w, s, slab)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float(), w.float(), None, s, 0)
    assert rel_err(y, ref) < 1e-2
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, K)
    assert torch.isfinite(slab[:rows]).all(), "statistics rows left unwritten"
    assert rel_err(slab[:rows, 0].sum(0), yf.sum(0)) < 1e-3
    assert rel_err(slab[:rows, 1].sum(0), (yf * yf).sum(0)) < 1e-3
    # the replaced 128-tile kernel: same MFMA sequence per element -> identical bf16 output
    lib.mi_set_panel(0)
    lib.mi_set_nt_split_blocks(0)  # the unsplit k-order
    rows0 = lib.mi_conv_stat_rows_g(N, H, H, C, K, 1, 1, s, 0, P, P)
    y0 = _fwd(lib, x, w, s, torch.empty(rows0, 2, K, device="cuda"))
    lib.mi_set_nt_split_blocks(128)
    lib.mi_set_panel(2)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    # no statistics requested: the plain store path
    y2 = _fwd(lib, x, w, s, None)
    torch.cuda.synchronize()
    assert torch.equal(y2, y)
