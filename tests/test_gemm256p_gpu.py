"""Persistent 256x256 NT GEMM (csrc/kernels/gemm256p.hip: tiles chained into one k-step pipeline,
the previous tile's epilogue stored from registers under the next tile's first k-step) against an
fp32 PyTorch reference and against the non-persistent gemm256 kernel: ragged M / N / K, bias, tile
counts below / at / above one per CU, and the ViT-B/16 shapes."""
import pytest
import torch

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


@pytest.fixture(scope="module", autouse=True)
def _native():
    from mi355x_dp.ops import _lib
    _lib.load(True)
    torch.manual_seed(0)
    yield
    _lib.call("mi_set_gemm_persist", 0)


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6))


def _persist(A, B, C, bias):
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    M, K = A.shape
    N = B.shape[0]
    _lib.call("mi_set_gemm_persist", 1)
    rc = _lib.load().mi_gemm256p_nt(ptr(A), ptr(B), ptr(C), ptr(bias), ptr(None), 0, M, N, K, K, K, N, stream_of(A))
    torch.cuda.synchronize()
    return rc


def _plain(A, B, C, bias):
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    M, K = A.shape
    N = B.shape[0]
    _lib.call("mi_set_gemm_persist", 0)
    _lib.call("mi_gemm256_nt", ptr(A), ptr(B), ptr(C), ptr(bias), ptr(None), 0, M, N, K, K, K, N, 0, 0, stream_of(A))
    torch.cuda.synchronize()


@pytest.mark.parametrize("M,N,K,use_bias", [
    (512, 512, 192, True),          # 4 tiles: fewer tiles than CUs, 3 k-steps (the minimum)
    (1000, 776, 200, True),         # ragged M / N / K
    (257, 264, 72 * 3, False),      # one row / 8 columns past a tile edge
    (50432, 2304, 768, True),       # ViT qkv forward: 1,773 tiles, ~7 per block
    (50432, 768, 3072, False),      # ViT fc1 data gradient: 591 tiles, 2-3 per block, long K
    (50432, 768, 768, False),       # ViT proj data gradient
    (256 * 256, 256, 256, True),    # exactly one tile per CU
])
def test_gemm256p_matches_reference_and_plain_kernel(M, N, K, use_bias):
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(BF)
    B = (torch.rand(N, K, device="cuda") * 2 - 1).to(BF)
    bias = torch.randn(N, device="cuda") if use_bias else None
    C = torch.full((M, N), float("nan"), dtype=BF, device="cuda")
    assert _persist(A, B, C, bias) == 0
    ref = A.float() @ B.float().t() + (bias if use_bias else 0)
    assert not torch.isnan(C).any()
    assert rel_err(C, ref) < 1e-2
    # the same fp32 accumulation order and rounding points as the non-persistent kernel without its
    # tail split-K (which sums a last partial wave's tiles in K slices): identical
    from mi355x_dp.ops import _lib
    C2 = torch.empty_like(C)
    _lib.call("mi_set_tail_split", 0)
    try:
        _plain(A, B, C2, bias)
    finally:
        _lib.call("mi_set_tail_split", 1)
    assert torch.equal(C, C2)


def test_gemm256p_declines_outside_contract():
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    A = torch.zeros(512, 128, dtype=BF, device="cuda")  # 2 k-steps: below the 3 the pipeline needs
    B = torch.zeros(512, 128, dtype=BF, device="cuda")
    C = torch.empty(512, 512, dtype=BF, device="cuda")
    _lib.call("mi_set_gemm_persist", 1)
    assert _lib.load().mi_gemm256p_nt(ptr(A), ptr(B), ptr(C), ptr(None), ptr(None), 0, 512, 512, 128, 128, 128, 512,
                                      stream_of(A)) != 0
    _lib.call("mi_set_gemm_persist", 0)
