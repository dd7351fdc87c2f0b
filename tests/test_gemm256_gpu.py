"""Deep-pipelined 256x256 NT GEMM (csrc/kernels/gemm256.hip) against an fp32 PyTorch reference:
ragged M / N / K, bias, fp32 and bf16 outputs, accumulate, and every fused epilogue op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


@pytest.fixture(scope="module", autouse=True)
def _native():
    from mi355x_dp.ops import _lib
    _lib.load(True)
    torch.manual_seed(0)


@pytest.fixture(params=[0, 2], ids=["bm256", "bm224"])
def bm224(request):
    """the NT kernel's row tile: 256 rows (mode 0) or forced 224 rows (mode 2; auto picks it where the
    wave quantization pays, gemm256.hip g256_wr)"""
    from mi355x_dp.ops import _lib
    lib = _lib.load()
    lib.mi_set_g256_bm224(request.param)
    yield request.param
    lib.mi_set_g256_bm224(1)


def test_gemm256_row_tile_choice():
    """auto mode (conv kernels): 224-row tiles for the 196-tile ResNet layer-3 / layer-4 grids, 256
    rows where the split tail already fills the chip"""
    from mi355x_dp.ops import _lib
    lib = _lib.load()
    lib.mi_set_g256_bm224(1)
    if torch.cuda.get_device_properties(0).multi_processor_count != 256:
        pytest.skip("cost model checked for 256 CUs")
    assert lib.mi_g256_stat_rows(50176, 256, 2304) == 2 * 224   # ceil(50176 / 224) tiles x 2 wave rows
    assert lib.mi_g256_stat_rows(12544, 512, 4608) == 2 * 56    # layer 4: 112 tiles, tail split 2
    assert lib.mi_g256_stat_rows(50432, 768, 3072) == 2 * 197  # 256 rows: tail split-K fills the chip


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6))


def run(A, B, C, bias=None, aux=None, epi=0, out_f32=0, acc=0):
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    M, K = A.shape
    N = B.shape[0]
    _lib.call("mi_gemm256_nt", ptr(A), ptr(B), ptr(C), ptr(bias), ptr(aux), epi, M, N, K, K, K, N, out_f32, acc,
              stream_of(A))
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,N,K", [(512, 512, 64), (1000, 776, 200), (50432 // 8, 3072, 768), (300, 256, 3072),
                                   (257, 264, 72), (4096, 4096, 4096)])
def test_gemm256_shapes(M, N, K, bm224):
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(BF)
    B = (torch.rand(N, K, device="cuda") * 2 - 1).to(BF)
    bias = torch.randn(N, device="cuda")
    ref = A.float() @ B.float().t() + bias
    C = torch.empty(M, N, dtype=BF, device="cuda")
    run(A, B, C, bias)
    assert rel_err(C, ref) < 1e-2
    Cf = torch.randn(M, N, device="cuda")
    base = Cf.clone()
    run(A, B, Cf, bias, out_f32=1, acc=1)
    assert rel_err(Cf, ref + base) < 1e-4


@pytest.mark.parametrize("epi", [1, 2, 3])
def test_gemm256_epilogues(epi, bm224):
    M, N, K = 600, 512, 256
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(BF)
    B = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.1).to(BF)
    aux = torch.randn(M, N, device="cuda").to(BF)
    C = torch.empty(M, N, dtype=BF, device="cuda")
    ref = (A.float() @ B.float().t()).to(BF).float()
    if epi == 1:
        u = torch.empty_like(C)
        run(A, B, C, aux=u, epi=1)
        x = ref.clone().requires_grad_()
        F.gelu(x).backward(torch.ones_like(x))
        assert rel_err(u, x.grad) < 1e-2          # aux = gelu'(pre-activation)
        assert rel_err(C, F.gelu(ref)) < 2e-2
    elif epi == 2:
        run(A, B, C, aux=aux, epi=2)               # C = acc * aux (aux: the stored derivative)
        assert rel_err(C, ref * aux.float()) < 2e-2
    else:
        run(A, B, C, aux=aux, epi=3)
        assert rel_err(C, ref + aux.float()) < 2e-2


@pytest.mark.parametrize("M,N,K", [(768, 3072, 50432 // 16), (2304, 768, 1000), (264, 136, 200), (512, 256, 64),
                                   (3072, 768, 6304)])
def test_gemm256_tn(M, N, K):
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    A = (torch.rand(K, M, device="cuda") * 2 - 1).to(BF)
    B = (torch.rand(K, N, device="cuda") * 2 - 1).to(BF)
    C = torch.randn(M, N, device="cuda")
    ref = C + A.float().t() @ B.float()
    _lib.call("mi_gemm256_tn", ptr(A), ptr(B), ptr(C), M, N, K, M, N, N, stream_of(A))
    torch.cuda.synchronize()
    assert rel_err(C, ref) < 1e-4


@pytest.mark.parametrize("Nb,H,C,K", [(4, 14, 1024, 256), (2, 14, 256, 1024), (3, 9, 512, 264)])
def test_conv_wgrad_on_gemm256_tn(Nb, H, C, K):
    """MI355X_DP_WGRAD256: a 1x1 stride-1 weight gradient routed to the 256x256 TN GEMM (split-K slabs)
    accumulates dy^T x into dw like the implicit-GEMM kernel (fp32 reference)"""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    lib = _lib.load()
    CL = torch.channels_last
    x = (torch.rand(Nb, C, H, H, device="cuda") * 2 - 1).to(BF).contiguous(memory_format=CL)
    dy = (torch.rand(Nb, K, H, H, device="cuda") * 2 - 1).to(BF).contiguous(memory_format=CL)
    dw0 = torch.randn(K, C, device="cuda")
    ref = dw0 + dy.float().permute(0, 2, 3, 1).reshape(-1, K).t() @ x.float().permute(0, 2, 3, 1).reshape(-1, C)
    outs = []
    for t in (0, 1):
        lib.mi_set_wgrad256(t)
        dw = dw0.clone()
        try:
            _lib.call("mi_conv2d_wgrad", ptr(x), ptr(dy), ptr(dw), Nb, H, H, C, K, 1, 1, 1, 0, H, H, stream_of(x))
            torch.cuda.synchronize()
        finally:
            lib.mi_set_wgrad256(0)
        outs.append(dw)
        assert rel_err(dw, ref) < 1e-4, t


@pytest.mark.parametrize("Nb,H,C,K", [(2, 14, 256, 512), (3, 18, 320, 576), (2, 28, 512, 1024)])
def test_ds_dgrad_scatter_on_gemm256(Nb, H, C, K, conv256_forced):
    """the stride-2 1x1 shortcut data gradient (even pixels only, flags bit 0) on the 256-wide kernel with
    its rows scattered into dx's even pixels (mi_gemm256_nt_scat2) matches fp32 at the even pixels and
    leaves the odd ones untouched, like the 128-tile class kernel it replaces"""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    lib = conv256_forced
    CL = torch.channels_last
    P = H // 2
    dy = (torch.rand(Nb, K, P, P, device="cuda") * 2 - 1).to(BF).contiguous(memory_format=CL)
    w = ((torch.rand(K, C, 1, 1, device="cuda") * 2 - 1) * 0.1).to(BF)
    wt = w.reshape(K, C).t().contiguous()  # [C][K]
    ref = F.conv_transpose2d(dy.float(), w.float(), stride=2, output_padding=1)  # [Nb, C, H, H]
    outs = []
    for on in (1, 0):
        lib.mi_set_ds256(on)
        dx = torch.full((Nb, C, H, H), 7.0, device="cuda").to(BF).contiguous(memory_format=CL)
        try:
            _lib.call("mi_conv2d_dgrad_ex4", ptr(dy), ptr(wt), ptr(dx), Nb, H, H, C, K, 1, 1, 2, 0, P, P, 0,
                      ptr(None), ptr(None), ptr(None), 0, ptr(None), 1, ptr(None), ptr(None), ptr(None),
                      stream_of(dy))
            torch.cuda.synchronize()
        finally:
            lib.mi_set_ds256(1)
        outs.append(dx)
        ev = dx[:, :, 0::2, 0::2]
        assert rel_err(ev, ref[:, :, 0::2, 0::2]) < 2e-2, on
        assert bool((dx[:, :, 1::2, :] == 7.0).all()) and bool((dx[:, :, :, 1::2] == 7.0).all()), on


CONV256 = [  # N, C, H, K, R, stride, pad
    (2, 64, 14, 256, 1, 1, 0), (2, 256, 14, 256, 3, 1, 1), (3, 128, 9, 512, 3, 2, 1), (2, 512, 7, 320, 1, 1, 0),
    (1, 64, 30, 256, 3, 1, 1)]


@pytest.fixture
def conv256_forced():
    from mi355x_dp.ops import _lib
    lib = _lib.load()
    lib.mi_set_conv256_min_tiles(1)
    lib.mi_set_conv256_min_k(0)
    yield lib
    lib.mi_set_conv256_min_tiles(96)
    lib.mi_set_conv256_min_k(512)


@pytest.mark.parametrize("shape", CONV256)
def test_conv256_fwd_stats_and_dgrad(shape, conv256_forced, bm224):
    """conv forward (+ BN statistics epilogue) and stride-1 dgrad (plain / accumulate / BN-backward
    epilogues) on the 256x256 kernel vs the 128x128 kernel and an fp32 reference"""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    lib = conv256_forced
    N, C, H, K, R, s, p = shape
    CL = torch.channels_last
    P = (H + 2 * p - R) // s + 1
    x = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(BF).contiguous(memory_format=CL)
    st = stream_of(x)
    M = N * P * P
    rows = lib.mi_conv_stat_rows(M, K, C, R * R)
    assert rows == 2 * ((M + 255) // 256 if bm224 == 0 else (M + 223) // 224)
    slab = torch.full((rows + 64, 2, K), float("nan"), device="cuda")
    y = torch.empty(N, K, P, P, dtype=BF, device="cuda", memory_format=CL)
    _lib.call("mi_conv2d_fwd", ptr(x), ptr(w), ptr(y), ptr(None), ptr(slab), N, H, H, C, K, R, R, s, p, P, P, 0, st)
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv2d(x.float(), w.float(), None, s, p)
    assert rel_err(y, ref) < 1e-2
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, K)
    assert rel_err(slab[:rows, 0].sum(0), yf.sum(0)) < 1e-3
    assert rel_err(slab[:rows, 1].sum(0), (yf * yf).sum(0)) < 1e-3
    if s != 1:
        return
    # dgrad: dx = conv_transpose(dy, w)
    dy = torch.randn(N, K, P, P, device="cuda").to(BF).contiguous(memory_format=CL)
    wt = torch.empty(C, R, R, K, dtype=BF, device="cuda")
    _lib.call("mi_conv_wtrans", ptr(w), ptr(wt), K, R * R, C, st)
    refdx = torch.nn.grad.conv2d_input(x.shape, w.float(), dy.float(), s, p)
    dx = torch.empty_like(x)
    _lib.call("mi_conv2d_dgrad", ptr(dy), ptr(wt), ptr(dx), N, H, H, C, K, R, R, s, p, P, P, st)
    torch.cuda.synchronize()
    assert rel_err(dx, refdx) < 1e-2
    if C < 256:
        return  # the dgrad output has C columns: only C >= 256 runs on the 256-wide tiles
    # epi 3: accumulate into an existing gradient
    base = torch.randn_like(x, dtype=torch.float32).to(BF).contiguous(memory_format=CL)
    acc = base.clone()
    _lib.call("mi_conv2d_dgrad_ex", ptr(dy), ptr(wt), ptr(acc), N, H, H, C, K, R, R, s, p, P, P, 3, ptr(acc),
              ptr(None), ptr(None), 0, ptr(None), st)
    torch.cuda.synchronize()
    assert rel_err(acc, refdx + base.float()) < 1e-2
    # epi 4: relu mask of the producing BN's output + its backward statistics
    ybn = torch.randn_like(x, dtype=torch.float32).to(BF).contiguous(memory_format=CL)
    xbn = torch.randn_like(x, dtype=torch.float32).to(BF).contiguous(memory_format=CL)
    mean = torch.randn(C, device="cuda") * 0.1
    r2 = lib.mi_dgrad_stat_rows(N, H, H, C, P, P, 1, K, R * R)
    slab2 = torch.full((r2 + 64, 2, C), float("nan"), device="cuda")
    dz = torch.empty_like(x)
    _lib.call("mi_conv2d_dgrad_ex", ptr(dy), ptr(wt), ptr(dz), N, H, H, C, K, R, R, s, p, P, P, 4, ptr(ybn),
              ptr(xbn), ptr(mean), 1, ptr(slab2), st)
    torch.cuda.synchronize()
    dzr = refdx * (ybn.float() > 0)
    assert rel_err(dz, dzr) < 1e-2
    dzf = dz.float().permute(0, 2, 3, 1).reshape(-1, C)
    xf = xbn.float().permute(0, 2, 3, 1).reshape(-1, C)
    assert rel_err(slab2[:r2, 0].sum(0), dzf.sum(0)) < 1e-3
    assert rel_err(slab2[:r2, 1].sum(0), (dzf * (xf - mean)).sum(0)) < 1e-3
