#!/usr/bin/env python
"""BatchNorm elementwise-pass microbenchmark at the ResNet-50 bs256 shapes: the forward apply
(y = relu(x*scale + shift [+ res])) and the backward apply (dx = k0*dz' + k1*x + k2 with the relu
mask, optional dres) timed alone, reported as achieved HBM bandwidth (bytes moved / time).

    python tools/bench_bn.py [--batch 256]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

BF = torch.bfloat16


def timeit(fn, iters=20):
    for _ in range(3):
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
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops._lib import ptr, stream_of
    _lib.load(True)
    dev = torch.device("cuda", 0)
    B = a.batch
    # (H*W, C) of the ResNet-50 BN layers at 224x224
    shapes = [(112 * 112, 64), (56 * 56, 64), (56 * 56, 256), (28 * 28, 128), (28 * 28, 512), (14 * 14, 256),
              (14 * 14, 1024), (7 * 7, 512), (7 * 7, 2048)]
    print("| M x C | pass | us | GB moved | TB/s |\n|---|---|---:|---:|---:|")
    tot_t = tot_b = 0.0
    for hw, C in shapes:
        M = B * hw
        x = torch.randn(M, C, device=dev).to(BF)
        res = torch.randn(M, C, device=dev).to(BF)
        y = torch.empty_like(x)
        g = torch.rand(C, device=dev) + 0.5
        bta = torch.randn(C, device=dev)
        rm = torch.randn(C, device=dev)
        rv = torch.rand(C, device=dev) + 0.5
        sc = torch.empty(C, device=dev)
        sh = torch.empty(C, device=dev)
        st = stream_of(x)
        for name, r in (("fwd apply", None), ("fwd apply +res", res)):
            f = lambda: _lib.call("mi_bn_fwd_eval", ptr(x), ptr(r), ptr(y), M, C, 1e-5, ptr(g), ptr(bta), ptr(rm),  # noqa
                                  ptr(rv), ptr(sc), ptr(sh), 1, st)
            t = timeit(f)
            nb = M * C * 2 * (3 if r is not None else 2)
            tot_t += t
            tot_b += nb
            print(f"| {M} x {C} | {name} | {t * 1e3:.1f} | {nb / 1e9:.3f} | {nb / t / 1e9:.2f} |")
        coef = torch.randn(3 * C, device=dev)
        mean = torch.randn(C, device=dev)
        inv = torch.rand(C, device=dev) + 0.5
        dg = torch.zeros(C, device=dev)
        db = torch.zeros(C, device=dev)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x)
        part = torch.zeros(2 * (1 + 64) * C, device=dev)
        for name, drs in (("bwd apply", None), ("bwd apply +dres", dres)):
            f = lambda: _lib.call("mi_bn_bwd_train_pre", ptr(x), ptr(res), ptr(dx), ptr(drs), M, C, ptr(g),  # noqa
                                  ptr(mean), ptr(inv), ptr(dg), ptr(db), ptr(coef), ptr(part), 1, st)
            t = timeit(f)
            nb = M * C * 2 * (4 if drs is not None else 3)
            tot_t += t
            tot_b += nb
            print(f"| {M} x {C} | {name} | {t * 1e3:.1f} | {nb / 1e9:.3f} | {nb / t / 1e9:.2f} |")
    print(f"\nall passes: {tot_t:.3f} ms, {tot_b / 1e9:.2f} GB, {tot_b / tot_t / 1e9:.2f} TB/s")


if __name__ == "__main__":
    main()
