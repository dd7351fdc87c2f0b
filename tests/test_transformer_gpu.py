"""Transformer kernels (csrc/kernels/transformer.hip + the NT GEMM epilogues) and the fused
ViT encoder layer against plain PyTorch fp32 references of the same ops."""
import math

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
    a = a.detach().float()
    b = b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(BF)


@pytest.mark.parametrize("M,D", [(300, 768), (77, 64), (5, 1024), (130, 200), (4099, 768), (33, 512)])
def test_layernorm_fwd_bwd(M, D):
    from mi355x_dp.ops import transformer as T
    x = rnd(M, D, scale=2.0) + 0.5
    w = torch.randn(D, device="cuda") * 0.5 + 1
    b = torch.randn(D, device="cuda") * 0.1
    y, mean, rstd = T._ln_fwd(x, w, b, 1e-6)
    xf = x.float().requires_grad_()
    wf, bf = w.clone().requires_grad_(), b.clone().requires_grad_()
    ref = F.layer_norm(xf, (D,), wf, bf, 1e-6)
    assert rel_err(y, ref) < 1e-2
    dy = rnd(M, D)
    dres = rnd(M, D)
    ref.backward(dy.float())
    dx, dw, db = T._ln_bwd(dy, x, w, b, mean, rstd, dres=dres)
    assert rel_err(dx, xf.grad + dres.float()) < 2e-2
    assert rel_err(dw, wf.grad) < 1e-2
    assert rel_err(db, bf.grad) < 1e-2


@pytest.mark.parametrize("M,N", [(1000, 768), (37, 2304), (4096, 8)])
def test_colsum(M, N):
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    x = rnd(M, N)
    out = torch.full((N,), 0.25, device="cuda")
    _lib.call("mi_colsum_bf16", ptr(x), ptr(out), M, N, N, stream_of(x))
    torch.cuda.synchronize()
    assert rel_err(out, x.float().sum(0) + 0.25) < 1e-4


@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm_epilogues(epi):
    from mi355x_dp.ops import transformer as T
    M, N, K = 333, 256, 192
    a, w = rnd(M, K), rnd(N, K, scale=0.1)
    bias = torch.randn(N, device="cuda") * 0.1
    aux = rnd(M, N)
    ref = a.float() @ w.float().t() + bias
    if epi == 1:
        out, u = T._gemm(a, w, bias, 1)
        x = ref.to(BF).float().requires_grad_()
        F.gelu(x).backward(torch.ones_like(x))
        assert rel_err(u, x.grad) < 1e-2           # aux = gelu'(pre-activation)
        ref = F.gelu(ref)
    else:
        out = T._gemm(a, w, bias, epi, aux if epi else None)
        if epi == 2:                               # C = acc * aux (the stored derivative)
            ref = ref.to(BF).float() * aux.float()
        elif epi == 3:
            ref = ref.to(BF).float() + aux.float()
    assert rel_err(out, ref) < 2e-2


def _block(D, heads, mlp):
    from mi355x_dp.models.vit import EncoderBlock
    torch.manual_seed(1)
    blk = EncoderBlock(heads, D, mlp)
    with torch.no_grad():  # non-trivial LN affine / biases
        for n, p in blk.named_parameters():
            if "ln" in n:
                p.add_(torch.randn_like(p) * 0.1)
            elif n.endswith("bias"):
                p.copy_(torch.randn_like(p) * 0.05)
    return blk


@pytest.mark.parametrize("B,T,D,heads,mlp", [(2, 17, 128, 4, 256), (3, 197, 768, 12, 3072)])
def test_encoder_layer_matches_fp32(B, T, D, heads, mlp):
    blk = _block(D, heads, mlp)
    x = (torch.randn(B, T, D) * 0.5).to(BF).float()
    dz = (torch.randn(B, T, D) * 0.1).to(BF).float()
    # fp32 reference: the module's unfused path on the host
    ref_blk = _block(D, heads, mlp)
    xr = x.clone().requires_grad_()
    zr = ref_blk(xr)
    zr.backward(dz)
    # native fused layer
    blk = blk.cuda()
    xg = x.cuda().to(BF).requires_grad_()
    zg = blk(xg)
    assert zg.dtype == BF
    zg.backward(dz.cuda().to(BF))
    torch.cuda.synchronize()
    assert rel_err(zg.cpu(), zr) < 3e-2
    assert rel_err(xg.grad.cpu(), xr.grad) < 5e-2
    for (n, p), (_, pr) in zip(blk.named_parameters(), ref_blk.named_parameters()):
        assert p.grad is not None, n
        assert rel_err(p.grad.cpu(), pr.grad) < 6e-2, n


def test_vit_native_forward_backward_small():
    from mi355x_dp.models.vit import VisionTransformer
    torch.manual_seed(0)
    m = VisionTransformer(image_size=32, patch_size=16, num_layers=2, num_heads=4, hidden_dim=64, mlp_dim=128,
                          num_classes=10).cuda()
    x = torch.randn(4, 3, 32, 32, device="cuda")
    out = m(x)
    loss = F.cross_entropy(out.float(), torch.arange(4, device="cuda"))
    loss.backward()
    assert math.isfinite(loss.item())
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


@pytest.mark.parametrize("B,T,H", [(2, 197, 12), (3, 17, 2), (1, 64, 4), (2, 250, 3), (4, 1, 1)])
def test_attention_fwd_bwd(B, T, H):
    from mi355x_dp.ops import transformer as Tm
    D = H * 64
    qkv = rnd(B * T, 3 * D, scale=1.5)
    do = rnd(B * T, D)
    x = qkv.clone().requires_grad_()
    o = Tm.attention(x, B, T, H)
    o.backward(do)
    xr = qkv.float().requires_grad_()
    q, k, v = xr.view(B, T, 3, H, 64).permute(2, 0, 3, 1, 4).unbind(0)
    orf = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B * T, D)
    orf.backward(do.float())
    assert rel_err(o, orf) < 2e-2
    dq, dr = x.grad.view(B * T, 3, D), xr.grad.view(B * T, 3, D)
    for i, name in enumerate("qkv"):
        if float(dr[:, i].abs().max()) < 1e-4:  # T == 1: dQ, dK are exactly zero
            assert float(dq[:, i].float().abs().max()) < 1e-4, name
        else:
            assert rel_err(dq[:, i], dr[:, i]) < 4e-2, name


@pytest.mark.parametrize("B,T,H", [(2, 197, 12), (3, 17, 2), (2, 224, 3), (4, 1, 1)])
def test_attention_fused_bwd_matches_two_kernels(B, T, H):
    """The single-kernel backward (dQ pass, then dK/dV pass in the same workgroup) against the dQ +
    dK/dV kernel pair: the same MFMA / exp sequence per element, so bit-identical."""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import transformer as Tm
    D = H * 64
    qkv = rnd(B * T, 3 * D, scale=1.5)
    do = rnd(B * T, D)
    grads = []
    try:
        for fused in (1, 0):
            _lib.call("mi_set_att_fused_bwd", fused)
            x = qkv.clone().requires_grad_()
            Tm.attention(x, B, T, H).backward(do)
            torch.cuda.synchronize()
            grads.append(x.grad.clone())
    finally:
        _lib.call("mi_set_att_fused_bwd", 1)
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("B,T,H", [(2, 197, 12), (3, 17, 2), (2, 256, 3), (4, 1, 1), (1, 100, 2)])
def test_attention_fwd_variants_agree(B, T, H):
    """The 8-wave online-softmax forward against the 4-wave single-pass forward: O and the saved
    log-sum-exp agree to rounding."""
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    D = H * 64
    qkv = rnd(B * T, 3 * D, scale=2.0)
    outs = []
    try:
        for waves in (4, 8):
            _lib.call("mi_set_att_fwd_waves", waves)
            o = torch.empty(B * T, D, dtype=BF, device="cuda")
            lse = torch.empty(B * H * T, device="cuda")
            _lib.call("mi_attn_fwd", ptr(qkv), ptr(o), ptr(lse), B, T, H, 0.125, stream_of(qkv))
            torch.cuda.synchronize()
            outs.append((o.float(), lse))
    finally:
        _lib.call("mi_set_att_fwd_waves", 8)
    for o, lse in outs[1:]:
        assert rel_err(o, outs[0][0]) < 1e-2
        assert float((lse - outs[0][1]).abs().max()) < 1e-4


def test_vit_native_matches_cpu_fp32():
    """The GPU ViT step -- native token embedding (class token + position embedding in one pass,
    fixed-order batch sums in backward) and the class-token-only final LayerNorm -- against the same
    module's stock fp32 CPU path (torch.cat, broadcast add, full-sequence LayerNorm)."""
    import copy
    from mi355x_dp.models.vit import VisionTransformer
    torch.manual_seed(0)
    m = VisionTransformer(image_size=64, patch_size=16, num_layers=2, num_heads=1, hidden_dim=64, mlp_dim=128,
                          num_classes=10)
    with torch.no_grad():  # the zero-initialised head / class token would make the check trivial
        m.heads.head.weight.normal_(std=0.2)
        m.class_token.normal_(std=0.5)
    mc = copy.deepcopy(m)
    mg = m.cuda()
    x = torch.randn(6, 3, 64, 64)
    y = torch.arange(6) % 10
    out_g = mg(x.cuda())
    out_c = mc(x)
    assert rel_err(out_g.float().cpu(), out_c) < 5e-2
    F.cross_entropy(out_g.float(), y.cuda()).backward()
    F.cross_entropy(out_c, y).backward()
    for name in ("class_token", "encoder.pos_embedding", "conv_proj.weight", "conv_proj.bias", "encoder.ln.weight",
                 "encoder.ln.bias", "heads.head.weight"):
        gg = mg.get_parameter(name).grad
        gc = mc.get_parameter(name).grad
        assert gg is not None, name
        assert rel_err(gg.float().cpu(), gc) < 8e-2, (name, rel_err(gg.float().cpu(), gc))
