"""Workspaces vs captured HIP graphs.

A HIP graph bakes in the device pointers of every workspace its kernels used at capture time: the
split-K slabs (gemm_conv.hip), the LayerNorm parameter-gradient replicas (transformer.hip) and the
gemm256 tail split-K partials (gemm256.hip).  When a later launch grows one of them the old buffer
must stay allocated (common.h ``mi_ws_retire``) or the earlier graph replays into freed memory.

The test captures one launch of each (plus an NT split-K GEMM), replays, grows every workspace on
the same slot far past its size, scribbles over freshly allocated memory, replays again, and
requires both replays to equal the eager launches bit for bit (the LayerNorm parameter
gradients, summed by fp32 atomics, to rounding)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(*shape, dtype=torch.bfloat16):
        return (torch.randn(*shape, device="cuda", generator=g) * 0.5).to(dtype)

    # TN split-K through slabs: C[128][128] += A[K][128]^T B[K][128], K large, one tile
    Kt = 65536
    ta, tb = rnd(Kt, 128), rnd(Kt, 128)
    tc = torch.zeros(128, 128, device="cuda")
    # NT split-K (small grid): 256 x 128 output, K = 8192
    na, nb = rnd(256, 8192), rnd(128, 8192)
    nc = torch.empty(256, 128, device="cuda", dtype=torch.bfloat16)
    # LayerNorm backward with parameter-gradient replicas
    M, D = 4096, 768
    lx, ldy = rnd(M, D), rnd(M, D)
    lw = torch.rand(D, device="cuda", generator=g) + 0.5
    lmean = torch.randn(M, device="cuda", generator=g) * 0.1
    lrstd = torch.rand(M, device="cuda", generator=g) + 0.5
    ldx = torch.empty_like(lx)
    ldw, ldb = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
    # gemm256 with a split tail: 2048 x 768 (24 tiles < 3/4 of the CUs), K = 3072 (12 k-tiles per split)
    ga, gb = rnd(2048, 3072), rnd(768, 3072)
    gc = torch.empty(2048, 768, device="cuda", dtype=torch.bfloat16)

    def run():
        st = stream_of(tc)
        tc.zero_()
        ldw.zero_()
        ldb.zero_()
        _lib.call("mi_gemm_tn", ptr(ta), ptr(tb), ptr(tc), 128, 128, Kt, 128, 128, 128, st)
        _lib.call("mi_gemm_nt_epi", ptr(na), ptr(nb), ptr(nc), ptr(None), ptr(None), 0, 256, 128, 8192, 8192,
                  8192, 128, st)
        _lib.call("mi_layernorm_bwd", ptr(ldy), ptr(lx), ptr(lw), ptr(lmean), ptr(lrstd), ptr(None), ptr(ldx),
                  ptr(ldw), ptr(ldb), M, D, st)
        _lib.call("mi_gemm256_nt", ptr(ga), ptr(gb), ptr(gc), ptr(None), ptr(None), 0, 2048, 768, 3072, 3072,
                  3072, 768, 0, 0, st)
        return [t.clone() for t in (tc, nc, ldx, ldw, ldb, gc)]

    return run


def test_graph_replay_survives_workspace_growth():
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import stream_of
    run = _ops()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ref = run()  # eager on the capture stream: every workspace of these shapes allocated here
        ref2 = run()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(ref, ref2)):
        if i not in (3, 4):  # the LayerNorm parameter gradients are atomically summed
            assert torch.equal(a, b)  # deterministic schedules
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        outs = run()
    g.replay()
    torch.cuda.synchronize()
    first = [o.clone() for o in outs]
    # grow every workspace of the capture stream's slots far past what the graph baked in
    lib = _lib.load(True)
    with torch.cuda.stream(s):
        h = stream_of()
        assert lib.mi_splitk_ws_reserve(256 << 20, h) == 0
        assert lib.mi_ln_ws_reserve(8192, h) == 0
        assert lib.mi_g256_tail_ws_reserve(64 << 20, 4096, h) == 0, "the tail split did not run on this stream"
    torch.cuda.synchronize()
    junk = [torch.full((64 << 20,), float("nan"), device="cuda") for _ in range(4)]  # reuse freed memory
    g.replay()
    torch.cuda.synchronize()
    del junk
    names = ("tn_splitk", "nt_splitk", "ln_dx", "ln_dw", "ln_db", "gemm256_tail")
    for name, a, b, c in zip(names, ref, first, outs):
        if name in ("ln_dw", "ln_db"):  # replicas summed by fp32 atomics: order-dependent rounding
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-4), name
            assert torch.allclose(a, c, rtol=1e-5, atol=1e-4), f"{name}: replay after workspace growth differs"
            continue
        assert torch.equal(a, b), name
        assert torch.equal(a, c), f"{name}: replay after workspace growth differs"
