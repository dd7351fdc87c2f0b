"""Fused ResNet stem (mi355x_dp.ops.stem: conv -> BN -> ReLU -> maxpool as one node, BN+ReLU
applied inside the pool, mask recomputed in backward) against the per-op native path and an fp32
PyTorch reference of the same ops."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6))


def _modules(seed=0):
    from mi355x_dp.models.layers import BatchNorm2d, Conv2d, MaxPool2d
    torch.manual_seed(seed)
    conv = Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
    bn = BatchNorm2d(64)
    with torch.no_grad():
        bn.weight.uniform_(-1.5, 1.5)  # negative scales: the pool must take max AFTER the affine
        bn.bias.uniform_(-0.3, 0.3)
    return conv.cuda(), bn.cuda(), MaxPool2d(3, 2, 1)


@pytest.mark.parametrize("n,size", [(16, 64), (4, 224), (8, 57)])
def test_fused_stem_matches_per_op(n, size):
    from mi355x_dp.models.layers import conv_bn, to_device_input
    from mi355x_dp.ops import stem as S
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(n, 3, size, size, device="cuda", generator=g)
    conv, bn, pool = _modules()
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    xi = to_device_input(x)
    assert S.fusable(conv, bn, pool, xi)
    y_f = S.stem(conv, bn, pool, xi)
    y_p = pool(conv_bn(conv2, bn2, xi, relu=True))
    assert y_f.shape == y_p.shape
    assert torch.equal(y_f, y_p)  # same bf16 values, same arg-max routing
    for a, b in ((bn.running_mean, bn2.running_mean), (bn.running_var, bn2.running_var)):
        assert rel_err(a, b) < 1e-5
    assert int(bn.num_batches_tracked) == int(bn2.num_batches_tracked) == 1
    dy = torch.randn(y_f.shape, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y_f.backward(dy)
    y_p.backward(dy)
    torch.cuda.synchronize()
    # fp32 reference of the same ops from the same (bf16-rounded) input and weights
    xr = xi[:, :3].float()
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_()
    gr, br = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    ref = F.max_pool2d(F.relu(F.batch_norm(F.conv2d(xr, wr, None, 2, 3), None, None, gr, br, True, 0.1, bn.eps)),
                       3, 2, 1)
    ref.backward(dy.float())
    for name, fused, per_op, r in (("conv", conv.weight.grad, conv2.weight.grad, wr.grad),
                                   ("gamma", bn.weight.grad, bn2.weight.grad, gr.grad),
                                   ("beta", bn.bias.grad, bn2.bias.grad, br.grad)):
        e_f, e_p = rel_err(fused, r), rel_err(per_op, r)
        assert e_f <= 1.25 * e_p + 0.01, (name, e_f, e_p)
        assert rel_err(fused, per_op) < 3e-2, name


@pytest.mark.parametrize("k,r,stride,pad", [(64, 3, 1, 1), (32, 7, 2, 3), (64, 5, 2, 2)])
def test_fused_stem_other_geometries(k, r, stride, pad):
    """fusable() accepts any small-channel bias-free stem: the persistent 7x7/2/64 weight-gradient
    kernel must refuse the others and the generic path must give the right gradient
    without touching other parameters' slices of the flat gradient buffer"""
    from mi355x_dp.models.layers import BatchNorm2d, Conv2d, MaxPool2d, conv_bn, to_device_input
    from mi355x_dp.ops import stem as S
    torch.manual_seed(1)
    conv = Conv2d(3, k, kernel_size=r, stride=stride, padding=pad, bias=False).cuda()
    bn = BatchNorm2d(k).cuda()
    pool = MaxPool2d(3, 2, 1)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    g = torch.Generator(device="cuda").manual_seed(5)
    xi = to_device_input(torch.randn(4, 3, 40, 40, device="cuda", generator=g))
    assert S.fusable(conv, bn, pool, xi)
    # sentinel gradient buffers around the conv's: a wrong-geometry kernel would write past it
    conv.weight.grad = torch.zeros_like(conv.weight)
    y = S.stem(conv, bn, pool, xi)
    y_p = pool(conv_bn(conv2, bn2, xi, relu=True))  # per-op native path: same bf16 rounding points
    dy = torch.randn(y.shape, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y.backward(dy)
    y_p.backward(dy)
    torch.cuda.synchronize()
    xr = xi[:, :3].float()
    wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_()
    gr, br = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    ref = F.max_pool2d(F.relu(F.batch_norm(F.conv2d(xr, wr, None, stride, pad), None, None, gr, br, True, 0.1,
                                           bn.eps)), 3, 2, 1)
    assert rel_err(y, ref) < 2e-2
    ref.backward(dy.float())
    assert conv.weight.grad.shape == wr.grad.shape
    # against fp32: no worse than the per-op native path (bf16 activations, BN backward at M=6400
    # amplifies their rounding), and close to that path itself
    for name, fused, per_op, ref_g in (("conv", conv.weight.grad, conv2.weight.grad, wr.grad),
                                       ("gamma", bn.weight.grad, bn2.weight.grad, gr.grad),
                                       ("beta", bn.bias.grad, bn2.bias.grad, br.grad)):
        e_f, e_p = rel_err(fused, ref_g), rel_err(per_op, ref_g)
        assert e_f <= 1.25 * e_p + 0.01, (name, e_f, e_p)
        assert rel_err(fused, per_op) < 3e-2, name


def test_fused_stem_used_in_resnet():
    from mi355x_dp.models import resnet50
    from mi355x_dp.ops import cross_entropy
    import mi355x_dp.models.resnet as R
    assert R.FUSED_STEM
    m = resnet50(num_classes=10).cuda()
    x = torch.randn(2, 3, 64, 64, device="cuda")
    out = m(x)
    assert type(out.grad_fn).__name__ != "", out.grad_fn
    # walk back to the stem: the graph must contain the fused node, not a max-pool node
    seen, stack = set(), [out.grad_fn]
    while stack:
        f = stack.pop()
        if f is None or f in seen:
            continue
        seen.add(f)
        stack.extend(nf for nf, _ in f.next_functions)
    names = {type(f).__name__ for f in seen}
    assert "_StemBackward" in names and "_MaxPoolBackward" not in names, names
    cross_entropy(out, torch.tensor([1, 2], device="cuda")).backward()
    assert m.conv1.weight.grad is not None and m.bn1.weight.grad.abs().sum() > 0


@pytest.mark.parametrize("n,size", [(40, 58), (2, 224), (3, 33)])
def test_stem_conv_kernel_and_stats(n, size):
    """persistent LDS-ring stem conv (7x7/2, 8-channel input, 64 outputs): output vs fp32 conv and
    its per-block BN statistics rows vs sums over the bf16 output; (40, 58): odd output rows and
    blocks whose pair range crosses image boundaries (fresh ring loads)."""
    from mi355x_dp.models.layers import to_device_input
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops.functional import conv2d_with_stats
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(7)
    x = to_device_input(torch.randn(n, 3, size, size, device="cuda", generator=g))
    w = (torch.randn(64, 3, 7, 7, device="cuda", generator=g) * 0.1).to(torch.bfloat16).float()
    P = (size + 6 - 7) // 2 + 1
    assert lib.mi_stem_conv_ok(8, 64, 7, 7, 2, 3, P)
    y, (slab, rows) = conv2d_with_stats(x, w, 2, 3)
    torch.cuda.synchronize()
    ref = F.conv2d(x[:, :3].float(), w, None, 2, 3)
    assert rel_err(y, ref) < 1e-2
    yf = y.float()
    s = slab[:rows].sum(0)
    assert torch.allclose(s[0], yf.sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)
    assert torch.allclose(s[1], (yf * yf).sum(dim=(0, 2, 3)), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("n,size", [(40, 58), (2, 224), (3, 33)])
def test_stem_wgrad_kernel(n, size):
    """persistent stem weight-gradient kernel (transposed LDS reads of dy and of the input ring,
    per-block partials added atomically) vs the fp32 weight gradient of the same conv"""
    from mi355x_dp.models.layers import to_device_input
    from mi355x_dp.ops import conv2d
    g = torch.Generator(device="cuda").manual_seed(9)
    x = to_device_input(torch.randn(n, 3, size, size, device="cuda", generator=g))
    w = (torch.randn(64, 3, 7, 7, device="cuda", generator=g) * 0.1).to(torch.bfloat16).float()
    w = w.contiguous(memory_format=torch.channels_last).requires_grad_()
    y = conv2d(x, w, None, 2, 3)
    dy = torch.randn(y.shape, device="cuda", generator=g).to(torch.bfloat16)
    y.backward(dy.contiguous(memory_format=torch.channels_last))
    wr = w.detach().clone().requires_grad_()
    F.conv2d(x[:, :3].float(), wr, None, 2, 3).backward(dy.float())
    assert rel_err(w.grad, wr.grad) < 1e-2
