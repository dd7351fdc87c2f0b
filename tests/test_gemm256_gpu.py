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
def test_gemm256_shapes(M, N, K):
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
def test_gemm256_epilogues(epi):
    M, N, K = 600, 512, 256
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(BF)
    B = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.1).to(BF)
    aux = torch.randn(M, N, device="cuda").to(BF)
    C = torch.empty(M, N, dtype=BF, device="cuda")
    ref = (A.float() @ B.float().t()).to(BF).float()
    if epi == 1:
        u = torch.empty_like(C)
        run(A, B, C, aux=u, epi=1)
        assert rel_err(u, ref) < 1e-2
        assert rel_err(C, F.gelu(ref)) < 2e-2
    elif epi == 2:
        run(A, B, C, aux=aux, epi=2)
        x = aux.float().requires_grad_()
        F.gelu(x).backward(torch.ones_like(x))
        assert rel_err(C, ref * x.grad) < 2e-2
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
