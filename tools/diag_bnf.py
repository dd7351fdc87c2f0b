#!/usr/bin/env python
"""Diagnostics for the fp32 training BatchNorm (fp32.hip): forward statistics, apply, backward
coefficients and dx of one shape against fp64, printed per stage.

    python tools/diag_bnf.py [--relu 1 --res 1]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

CL = torch.channels_last


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(b.norm(), 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--relu", type=int, default=1)
    ap.add_argument("--res", type=int, default=1)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    lib = _lib.load(True)
    N, C, H = 32, 64, 16
    g = torch.Generator().manual_seed(2)
    x = torch.randn(N, C, H, H, generator=g, dtype=torch.float64) * 2 + 0.5
    r = torch.randn(N, C, H, H, generator=g, dtype=torch.float64)
    gamma = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    beta = torch.randn(C, generator=g, dtype=torch.float64)
    dy = torch.randn(N, C, H, H, generator=g, dtype=torch.float64)
    x32 = x.float().double()
    M = N * H * H
    xm = x32.permute(0, 2, 3, 1).reshape(M, C)
    rm_ = r.float().double().permute(0, 2, 3, 1).reshape(M, C)
    dym = dy.float().double().permute(0, 2, 3, 1).reshape(M, C)
    mean = xm.mean(0)
    var = xm.var(0, unbiased=False)
    invstd = 1.0 / torch.sqrt(var + 1e-5)
    pre = (xm - mean) * invstd * gamma + beta + (rm_ if a.res else 0)
    yref = pre.clamp_min(0) if a.relu else pre
    dz = dym * (yref > 0) if a.relu else dym
    xhat = (xm - mean) * invstd
    dxref = gamma * invstd * (dz - dz.mean(0) - xhat * (dz * xhat).mean(0))

    dev = "cuda"
    xc = x.float().to(dev).contiguous(memory_format=CL)
    rc = r.float().to(dev).contiguous(memory_format=CL) if a.res else None
    gc, bc = gamma.float().to(dev), beta.float().to(dev)
    part = torch.empty((lib.mi_f32_bn_partial_rows(M, C), 2, C), device=dev)
    sm, si, sc, sh = (torch.empty(C, device=dev) for _ in range(4))
    y = torch.empty_like(xc)
    rmn, rvr = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    nbt = torch.zeros((), dtype=torch.int64, device=dev)
    st = stream_of(xc)
    _lib.call("mi_f32_bn_fwd_train", ptr(xc), ptr(rc), ptr(y), M, C, 1e-5, 0.1, ptr(gc), ptr(bc), ptr(rmn), ptr(rvr),
              ptr(nbt), ptr(sm), ptr(si), ptr(sc), ptr(sh), ptr(part), a.relu, st)
    torch.cuda.synchronize()
    ym = y.permute(0, 2, 3, 1).reshape(M, C).double().cpu()
    print("mean", rel(sm, mean), "invstd", rel(si, invstd), "y", rel(ym, yref))
    mask_dis = int(((ym > 0) != (yref > 0)).sum())
    print("mask disagreements", mask_dis, "of", M * C)
    dyc = dy.float().to(dev).contiguous(memory_format=CL)
    coef = torch.empty((3, C), device=dev)
    dx = torch.empty_like(xc)
    dres = torch.empty_like(xc) if a.res else None
    gw, gb = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    part2 = torch.empty_like(part)
    _lib.call("mi_f32_bn_bwd_train", ptr(dyc), ptr(y), ptr(xc), ptr(dx), ptr(dres), M, C, ptr(gc), ptr(sm), ptr(si),
              ptr(gw), ptr(gb), ptr(coef), ptr(part2), a.relu, st)
    torch.cuda.synchronize()
    dxm = dx.permute(0, 2, 3, 1).reshape(M, C).double().cpu()
    print("dx", rel(dxm, dxref), "dbeta", rel(gb, dz.sum(0)), "dgamma", rel(gw, (dz * xhat).sum(0)))
    if a.res:
        print("dres", rel(dres.permute(0, 2, 3, 1).reshape(M, C), dz))
    err = (dxm - dxref).abs()
    print("dx err per channel (first 8):", [round(float(v), 5) for v in err.max(0).values[:8]])
    rows = err.max(1).values
    bad = (rows > 1e-3).nonzero().flatten()
    print("rows with err > 1e-3:", int(bad.numel()), "first:", bad[:16].tolist())
    bad_c = (err.max(0).values > 1e-3).nonzero().flatten()
    print("channels with err > 1e-3:", bad_c.tolist()[:32])
    # partial-slab readback: the backward slab (sum dz, sum dz (x - mean)) of block 0
    p0 = part2[0].double().cpu()
    rpb = M // part2.shape[0]
    print("rpb", rpb, "nblk", part2.shape[0])
    ref_s = dz[:rpb].sum(0)
    print("block0 sum dz rel", rel(p0[0], ref_s))


if __name__ == "__main__":
    main()
