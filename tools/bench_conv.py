#!/usr/bin/env python
"""Per-shape conv microbenchmark: every distinct conv of a ResNet (fwd / dgrad / wgrad)
timed on the native MFMA kernels and on stock PyTorch (MIOpen) bf16 channels_last,
reported as TFLOP/s.  Drives kernel tuning; writes a markdown table.

    python tools/bench_conv.py --model resnet50 --batch 256 [--no-stock]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

CL = torch.channels_last
BF = torch.bfloat16


def conv_shapes(model, batch, size):
    from mi355x_dp.models import get_model
    m = get_model(model)
    shapes = {}
    hooks = []

    def hook(mod, inp, out):
        x = inp[0]
        key = (x.shape[1], x.shape[2], mod.out_channels, mod.kernel_size[0], mod.stride[0], mod.padding[0])
        shapes[key] = shapes.get(key, 0) + 1

    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d):
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m(torch.zeros(1, 3, size, size))
    return [(batch, *k, n) for k, n in shapes.items()]


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--no-stock", action="store_true")
    ap.add_argument("--stages", type=int, default=1, help="NT kernel LDS stages (1 or 2)")
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    _lib.load().mi_set_glds(1); _lib.load().mi_set_nt_stages(a.stages)

    tot = {"fwd": [0, 0], "dgrad": [0, 0], "wgrad": [0, 0]}
    print("| N C H K R s | count | fwd TF (ms) | dgrad TF (ms) | wgrad TF (ms) | roof ms (mem/mfma) | stock fwd/dgrad/wgrad TF |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    roof_tot = 0.0
    for (N, C, H, K, R, s, p, cnt) in conv_shapes(a.model, a.batch, a.size):
        P = (H + 2 * p - R) // s + 1
        flops = 2.0 * N * P * P * K * C * R * R
        # roofline: 2.3 PFLOP/s dense bf16 MFMA, 6 TB/s achievable HBM; activations read+written once
        act = 2.0 * (N * H * H * C + N * P * P * K)
        t_mem, t_mma = act / 6e9, flops / 2.3e12
        roof = max(t_mem, t_mma)
        roof_tot += 3 * roof * cnt
        x = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(BF).contiguous(memory_format=CL)
        dy = torch.randn(N, K, P, P, device="cuda").to(BF).contiguous(memory_format=CL)
        res = {}
        st = stream_of(x)
        if C % 64 == 0:
            y = torch.empty(N, K, P, P, dtype=BF, device="cuda", memory_format=CL)
            res["fwd"] = timeit(lambda: _lib.call("mi_conv2d_fwd", ptr(x), ptr(w), ptr(y), ptr(None), ptr(None), N, H, H, C, K,
                                                  R, R, s, p, P, P, 0, st))
            wt = torch.empty(C, R, R, K, dtype=BF, device="cuda")
            dx = torch.empty_like(x)

            def dg():
                _lib.call("mi_conv_wtrans", ptr(w), ptr(wt), K, R * R, C, st)
                _lib.call("mi_conv2d_dgrad", ptr(dy), ptr(wt), ptr(dx), N, H, H, C, K, R, R, s, p, P, P, st)
            res["dgrad"] = timeit(dg)
            dw = torch.zeros(K, R, R, C, dtype=torch.float32, device="cuda")
            res["wgrad"] = timeit(lambda: _lib.call("mi_conv2d_wgrad", ptr(x), ptr(dy), ptr(dw), N, H, H, C, K, R,
                                                    R, s, p, P, P, st))
        stock = ""
        if not a.no_stock:
            xs = x.detach().requires_grad_()
            ws = w.detach().requires_grad_()
            tf = timeit(lambda: F.conv2d(xs, ws, None, s, p))
            td = timeit(lambda: torch.ops.aten.convolution_backward(dy, xs, ws, None, [s, s], [p, p], [1, 1], False,
                                                                   [0, 0], 1, [True, False, False]))
            tw = timeit(lambda: torch.ops.aten.convolution_backward(dy, xs, ws, None, [s, s], [p, p], [1, 1], False,
                                                                   [0, 0], 1, [False, True, False]))
            stock = f"{flops / tf / 1e9:.0f} / {flops / td / 1e9:.0f} / {flops / tw / 1e9:.0f}"
        cells = []
        for k in ("fwd", "dgrad", "wgrad"):
            if k in res:
                cells.append(f"{flops / res[k] / 1e9:.0f} ({res[k]:.3f})")
                tot[k][0] += res[k] * cnt
                tot[k][1] += flops * cnt
            else:
                cells.append("im2col")
        print(f"| {N} {C} {H} {K} {R} {s} | {cnt} | {cells[0]} | {cells[1]} | {cells[2]} | {t_mem:.3f}/{t_mma:.3f} | {stock} |", flush=True)
    for k, (t, f) in tot.items():
        print(f"\n**{k}**: {t:.2f} ms per step-equivalent, {f / t / 1e9:.0f} TFLOP/s aggregate")
    print(f"\n**roofline** (fwd+dgrad+wgrad, convs with C%64==0): {roof_tot:.2f} ms")


if __name__ == "__main__":
    main()
