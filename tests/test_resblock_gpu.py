"""Fused residual blocks (mi355x_dp.ops.resblock: one autograd node per block, BN-backward
statistics in the dgrad epilogue, in-place residual-gradient accumulation) against the per-op
native path on the same weights / inputs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6))


def _run(name, fused, x, y, seed=0):
    import mi355x_dp.models.resnet as R
    from mi355x_dp.models import get_model
    from mi355x_dp.ops import cross_entropy
    old = R.FUSED_BLOCKS
    R.FUSED_BLOCKS = fused
    try:
        torch.manual_seed(seed)
        m = get_model(name, num_classes=10).cuda()
        with torch.no_grad():  # non-trivial BN affine parameters
            for mod in m.modules():
                if isinstance(mod, torch.nn.BatchNorm2d):
                    mod.weight.uniform_(0.5, 1.5)
                    mod.bias.uniform_(-0.2, 0.2)
        # (the stem weight gradient depends on every block's input gradient, so the dx chain
        # through all blocks is covered without an input gradient)
        loss = cross_entropy(m(x), y)
        loss.backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}
        bufs = {n: b.detach().float().clone() for n, b in m.named_buffers()}
        return float(loss), grads, bufs
    finally:
        R.FUSED_BLOCKS = old


def _fp32_ref(name, x, y):
    """stock-PyTorch fp32 model (same architecture / names) with the same initial weights"""
    from mi355x_dp.models import get_model
    from mi355x_dp.models.stock import stock_resnet
    torch.manual_seed(0)
    m = get_model(name, num_classes=10)
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
    ref = stock_resnet(name, num_classes=10)
    ref.load_state_dict(m.state_dict())
    ref = ref.cuda().float()
    loss = torch.nn.functional.cross_entropy(ref(x), y)
    loss.backward()
    return float(loss), {n: p.grad.detach().float() for n, p in ref.named_parameters()}


@pytest.mark.parametrize("name,size", [("resnet18", 32), ("resnet50", 64), ("resnet34", 40)])
def test_fused_blocks_match_per_op(name, size):
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(8, 3, size, size, device="cuda", generator=g)
    y = torch.randint(0, 10, (8,), device="cuda", generator=g)
    l0, g0, b0 = _run(name, False, x, y)
    l1, g1, b1 = _run(name, True, x, y)
    lr, gr = _fp32_ref(name, x, y)
    assert l1 == pytest.approx(l0, rel=1e-3)
    for n in b0:
        assert rel_err(b1[n], b0[n]) < 1e-3, n
    worst = []
    for n in g0:
        e_per_op, e_fused = rel_err(g0[n], gr[n]), rel_err(g1[n], gr[n])
        worst.append((e_fused - e_per_op, n, e_fused, e_per_op))
        # fused must be as accurate as the per-op bf16 path (vs fp32), up to rounding noise
        assert e_fused <= 1.25 * e_per_op + 0.01, (n, e_fused, e_per_op)
    print(sorted(worst)[-3:])


@pytest.mark.parametrize("name,size,batch", [("resnet18", 224, 16), ("resnet50", 224, 32)])
def test_normalize_on_load_matches_materialised(name, size, batch, monkeypatch):
    """Inner BatchNorms normalized on load by their consumer convs (forward, weight gradient, ReLU
    mask from c in the data gradient; ops/resblock.py NOL) against the same fused blocks with the
    BN outputs materialised: losses / running statistics equal to rounding, every gradient as
    close to fp32 PyTorch as the materialised path, and the NOL path really taken (only layers
    whose grids do not split K take it: production-sized activations)."""
    import mi355x_dp.ops.resblock as RB
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(batch, 3, size, size, device="cuda", generator=g)
    y = torch.randint(0, 10, (batch,), device="cuda", generator=g)
    monkeypatch.setattr(RB, "NOL", False)
    l0, g0, b0 = _run(name, True, x, y)
    monkeypatch.setattr(RB, "NOL", True)
    used = RB.NOL_USED[0]
    l1, g1, b1 = _run(name, True, x, y)
    assert RB.NOL_USED[0] > used
    lr, gr = _fp32_ref(name, x, y)
    assert l1 == pytest.approx(l0, rel=2e-3)
    for n in b0:
        assert rel_err(b1[n], b0[n]) < 2e-3, n
    for n in g0:
        e_mat, e_nol = rel_err(g0[n], gr[n]), rel_err(g1[n], gr[n])
        assert e_nol <= 1.25 * e_mat + 0.01, (n, e_nol, e_mat)


@pytest.mark.parametrize("name,size,batch", [("resnet50", 224, 32)])
def test_folded_bn_backward_matches_materialised(name, size, batch, monkeypatch):
    """BatchNorm backward folded into its consumer convs' GEMMs (ops/resblock.py
    _Fold: the BN input gradient of 1x1 / stride-1 convs never materialised) against the same fused
    blocks with the materialised BN-backward apply: losses and running statistics equal, every
    gradient as close to fp32 PyTorch as the materialised path, and the folded path really taken."""
    import mi355x_dp.ops.resblock as RB
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(batch, 3, size, size, device="cuda", generator=g)
    y = torch.randint(0, 10, (batch,), device="cuda", generator=g)
    monkeypatch.setattr(RB, "BN_FOLD", False)
    used = RB.FOLD_USED[0]
    l0, g0, b0 = _run(name, True, x, y)
    assert RB.FOLD_USED[0] == used
    monkeypatch.setattr(RB, "BN_FOLD", True)
    l1, g1, b1 = _run(name, True, x, y)
    assert RB.FOLD_USED[0] > used
    lr, gr = _fp32_ref(name, x, y)
    assert l1 == l0  # the forward is untouched
    for n in b0:
        assert rel_err(b1[n], b0[n]) < 1e-3, n
    worst = []
    for n in g0:
        e_mat, e_fold = rel_err(g0[n], gr[n]), rel_err(g1[n], gr[n])
        worst.append((e_fold - e_mat, n, e_fold, e_mat))
        assert e_fold <= 1.25 * e_mat + 0.01, (n, e_fold, e_mat)
    print(sorted(worst)[-3:])


def test_fused_block_used_in_training():
    import mi355x_dp.models.resnet as R
    from mi355x_dp.models import get_model
    from mi355x_dp.ops import resblock
    m = get_model("resnet50").cuda()
    x = torch.randn(2, 3, 64, 64, device="cuda")
    assert R.FUSED_BLOCKS and resblock.fusable(m.layer1[0], torch.empty(1, device="cuda", dtype=torch.bfloat16))
    out = m.layer1[0](m.maxpool(R.conv_bn(m.conv1, m.bn1, R.to_device_input(x), relu=True)))
    assert type(out.grad_fn).__name__.startswith("_ResBlock")


@pytest.mark.parametrize("inpl,planes,stride,ds,size", [(256, 64, 1, False, 28), (256, 128, 2, True, 28),
                                                        (64, 64, 1, True, 16), (512, 256, 2, True, 14)])
def test_single_bottleneck_fused_vs_per_op(inpl, planes, stride, ds, size):
    """one block in isolation (well conditioned): input gradient, parameter gradients and BN
    running statistics of the fused node match the per-op native path to bf16 rounding"""
    import mi355x_dp.models.resnet as R
    from mi355x_dp.models.layers import BatchNorm2d
    res = {}
    g = torch.Generator(device="cuda").manual_seed(11)
    x0 = torch.randn(16, inpl, size, size, device="cuda", generator=g).to(torch.bfloat16)
    x0 = x0.contiguous(memory_format=torch.channels_last)
    dout = torch.randn(16, planes * 4, size // stride, size // stride, device="cuda", generator=g)
    for fused in (False, True):
        torch.manual_seed(3)
        down = torch.nn.Sequential(R.conv1x1(inpl, planes * 4, stride), BatchNorm2d(planes * 4)) if ds else None
        blk = R.Bottleneck(inpl, planes, stride, down).cuda()
        with torch.no_grad():
            for mod in blk.modules():
                if isinstance(mod, torch.nn.BatchNorm2d):
                    mod.weight.uniform_(0.5, 1.5)
                    mod.bias.uniform_(-0.2, 0.2)
        old = R.FUSED_BLOCKS
        R.FUSED_BLOCKS = fused
        try:
            x = x0.clone().requires_grad_()
            out = blk(x)
            assert (type(out.grad_fn).__name__ == "_ResBlockBackward") == fused
            out.backward(dout.to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        finally:
            R.FUSED_BLOCKS = old
        torch.cuda.synchronize()
        res[fused] = (out.float(), x.grad.float(), {n: p.grad.float() for n, p in blk.named_parameters()},
                      {n: b.float() for n, b in blk.named_buffers()})
    (o0, dx0, g0, b0), (o1, dx1, g1, b1) = res[False], res[True]
    assert rel_err(o1, o0) < 1e-2
    assert rel_err(dx1, dx0) < 2e-2
    for n in g0:
        assert rel_err(g1[n], g0[n]) < 2e-2, n
    for n in b0:
        assert rel_err(b1[n], b0[n]) < 1e-4, n


@pytest.mark.parametrize("force256", [False, True])
def test_block_chain_handoff_matches_per_op(force256):
    """three consecutive fused blocks (identity, downsample, identity): the cross-block hand-off
    (epilogue 5) is used and gradients match the per-op path.  The stride-2 shortcut's dgrad writes
    only the even pixels and conv1's dgrad reads the sum there only; force256 runs those dgrads on
    the 256x256 pipeline (its even-pixel epilogue) instead of the 128-tile kernel."""
    import mi355x_dp.models.resnet as R
    from mi355x_dp.models.layers import BatchNorm2d
    from mi355x_dp.ops import _lib, resblock
    lib = _lib.load()
    if force256:
        lib.mi_set_conv256_min_tiles(1)
        lib.mi_set_conv256_min_k(0)
    try:
        _chain_handoff(R, BatchNorm2d, resblock)
    finally:
        lib.mi_set_conv256_min_tiles(96)
        lib.mi_set_conv256_min_k(512)


def _chain_handoff(R, BatchNorm2d, resblock):
    g = torch.Generator(device="cuda").manual_seed(2)
    x0 = torch.randn(16, 256, 28, 28, device="cuda", generator=g).to(torch.bfloat16)
    x0 = x0.contiguous(memory_format=torch.channels_last)
    dout = torch.randn(16, 512, 14, 14, device="cuda", generator=g).to(torch.bfloat16)
    dout = dout.contiguous(memory_format=torch.channels_last)
    res = {}
    for fused in (False, True):
        torch.manual_seed(4)
        down = torch.nn.Sequential(R.conv1x1(256, 512, 2), BatchNorm2d(512))
        net = torch.nn.Sequential(R.Bottleneck(256, 64), R.Bottleneck(256, 128, 2, down),
                                  R.Bottleneck(512, 128)).cuda()
        with torch.no_grad():
            for mod in net.modules():
                if isinstance(mod, torch.nn.BatchNorm2d):
                    mod.weight.uniform_(0.5, 1.5)
                    mod.bias.uniform_(-0.2, 0.2)
        old = R.FUSED_BLOCKS
        R.FUSED_BLOCKS = fused
        used0 = resblock.HANDOFF_USED[0]
        try:
            x = x0.clone().requires_grad_()
            out = net(x)
            out.backward(dout)
        finally:
            R.FUSED_BLOCKS = old
        torch.cuda.synchronize()
        if fused:
            assert resblock.HANDOFF_USED[0] - used0 == 2   # blocks 1 and 2 receive hand-offs
            assert not resblock._HANDOFF                     # block 0's input is not a block output
        res[fused] = (x.grad.float(), {n: p.grad.float() for n, p in net.named_parameters()})
    (dx0, g0), (dx1, g1) = res[False], res[True]
    assert rel_err(dx1, dx0) < 2e-2
    for n in g0:
        assert rel_err(g1[n], g0[n]) < 2e-2, n


def test_abandoned_handoff_no_double_count():
    """A block output with a second consumer: the next block's conv1 dgrad still finalizes the
    previous block's last BatchNorm into scratch (hand-off), but the previous block receives the
    SUM of both consumers' gradients -- a different buffer -- so it must drop the hand-off and
    recompute; its affine gradients are then counted once (matches the per-op path)."""
    import mi355x_dp.models.resnet as R
    from mi355x_dp.ops import resblock
    g = torch.Generator(device="cuda").manual_seed(5)
    x0 = torch.randn(8, 256, 28, 28, device="cuda", generator=g).to(torch.bfloat16)
    x0 = x0.contiguous(memory_format=torch.channels_last)
    d_out = torch.randn(8, 256, 28, 28, device="cuda", generator=g).to(torch.bfloat16)
    d_mid = torch.randn(8, 256, 28, 28, device="cuda", generator=g).to(torch.bfloat16)
    res = {}
    for fused in (False, True):
        torch.manual_seed(6)
        b0, b1 = R.Bottleneck(256, 64).cuda(), R.Bottleneck(256, 64).cuda()
        with torch.no_grad():
            for mod in list(b0.modules()) + list(b1.modules()):
                if isinstance(mod, torch.nn.BatchNorm2d):
                    mod.weight.uniform_(0.5, 1.5)
                    mod.bias.uniform_(-0.2, 0.2)
        old = R.FUSED_BLOCKS
        R.FUSED_BLOCKS = fused
        used0 = resblock.HANDOFF_USED[0]
        try:
            x = x0.clone().requires_grad_()
            h = b0(x)
            out = b1(h)
            torch.autograd.backward([out, h], [d_out.contiguous(memory_format=torch.channels_last),
                                               d_mid.contiguous(memory_format=torch.channels_last)])
        finally:
            R.FUSED_BLOCKS = old
        torch.cuda.synchronize()
        if fused:
            assert resblock.HANDOFF_USED[0] == used0  # the hand-off was abandoned
        resblock._HANDOFF.clear()
        res[fused] = {n: p.grad.float() for n, p in list(b0.named_parameters()) + list(b1.named_parameters())}
    for n in res[False]:
        assert rel_err(res[True][n], res[False][n]) < 2e-2, n
