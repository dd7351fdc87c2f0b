#!/usr/bin/env python
"""Isolated A/B of the normalize-on-load kernels against the materialising schedule on the
ResNet-50 (batch 256) inner-BN shapes: forward (gather y vs normalize c on load), data gradient
(ReLU mask from y vs from c), weight gradient (y vs c normalized on load).  One process, rounds
interleaved, medians -- separates kernel cost from the in-model stream contention.

    python tools/bench_nol.py [--iters 20] [--batch 256]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mi355x_dp.ops import _lib
from mi355x_dp.ops._lib import ptr

BF16, F32 = torch.bfloat16, torch.float32
CL = torch.channels_last
EPI_BN_BWD = 4

# (name, C in, K out, H in, R, stride)
SHAPES = [
    ("l1.conv2 3x3", 64, 64, 56, 3, 1),
    ("l1.conv3 1x1", 64, 256, 56, 1, 1),
    ("l2.conv2 3x3 s2", 128, 128, 56, 3, 2),
    ("l2.conv2 3x3", 128, 128, 28, 3, 1),
    ("l2.conv3 1x1", 128, 512, 28, 1, 1),
    ("l3.conv2 3x3", 256, 256, 14, 3, 1),
    ("l3.conv3 1x1", 256, 1024, 14, 1, 1),
]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    lib = _lib.load(True)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    Nb = a.batch
    print("| shape | fwd y | fwd NoL | dgrad mask y | dgrad mask c | wgrad y | wgrad NoL | NoL ok |")
    print("|---|---:|---:|---:|---:|---:|---:|---|")
    for name, C, K, H, R, s in SHAPES:
        pad = R // 2
        P = (H + 2 * pad - R) // s + 1
        ok = bool(lib.mi_conv_nol_ok(Nb, H, H, C, K, R, R, s, pad, P, P))
        x = torch.randn(Nb, C, H, H, device=dev).to(BF16).contiguous(memory_format=CL)
        c = torch.randn(Nb, C, H, H, device=dev).to(BF16).contiguous(memory_format=CL)
        w = (torch.randn(K, R, R, C, device=dev) * 0.05).to(BF16).contiguous()  # [K][R][S][C]
        wt = (torch.randn(C, R, R, K, device=dev) * 0.05).to(BF16).contiguous()  # dgrad operand
        scale = torch.rand(C, device=dev) + 0.5
        shift = torch.randn(C, device=dev) * 0.1
        mean = torch.zeros(C, device=dev)
        y = torch.empty(Nb, K, P, P, dtype=BF16, device=dev, memory_format=CL)
        dy = torch.randn(Nb, K, P, P, device=dev).to(BF16).contiguous(memory_format=CL)
        dz = torch.empty(Nb, C, H, H, dtype=BF16, device=dev, memory_format=CL)
        g = torch.zeros(K, R, R, C, dtype=F32, device=dev)
        frows = lib.mi_conv_stat_rows_g(Nb, H, H, C, K, R, R, s, pad, P, P)
        fslab = torch.empty((frows + lib.mi_bn_slab_extra_rows(), 2, K), dtype=F32, device=dev)
        drows = lib.mi_dgrad_stat_rows(Nb, H, H, C, P, P, s, K, R * R)
        dslab = torch.empty((drows + lib.mi_bn_slab_extra_rows(), 2, C), dtype=F32, device=dev)

        def fwd_y():
            _lib.call("mi_conv2d_fwd", ptr(x), ptr(w), ptr(y), ptr(None), ptr(fslab), Nb, H, H, C, K, R, R, s, pad, P,
                      P, 0, st)

        def fwd_nol():
            _lib.call("mi_conv2d_fwd_nol", ptr(c), ptr(w), ptr(y), ptr(fslab), ptr(scale), ptr(shift), Nb, H, H, C, K,
                      R, R, s, pad, P, P, st)

        def dg_y():
            _lib.call("mi_conv2d_dgrad_ex2", ptr(dy), ptr(wt), ptr(dz), Nb, H, H, C, K, R, R, s, pad, P, P, EPI_BN_BWD,
                      ptr(x), ptr(c), ptr(mean), 1, ptr(dslab), 0, st)

        def dg_c():
            _lib.call("mi_conv2d_dgrad_ex3", ptr(dy), ptr(wt), ptr(dz), Nb, H, H, C, K, R, R, s, pad, P, P, EPI_BN_BWD,
                      ptr(None), ptr(c), ptr(mean), 1, ptr(dslab), 0, ptr(scale), ptr(shift), st)

        def wg_y():
            _lib.call("mi_conv2d_wgrad", ptr(x), ptr(dy), ptr(g), Nb, H, H, C, K, R, R, s, pad, P, P, st)

        def wg_nol():
            _lib.call("mi_conv2d_wgrad_nol", ptr(c), ptr(dy), ptr(g), ptr(scale), ptr(shift), Nb, H, H, C, K, R, R,
                      s, pad, P, P, st)

        fns = [fwd_y, fwd_nol, dg_y, dg_c, wg_y, wg_nol] if ok else [fwd_y, dg_y, wg_y]
        res = {f.__name__: [] for f in fns}
        for _ in range(a.rounds):
            for f in fns:
                res[f.__name__].append(timed(f, a.iters))
        med = {k: statistics.median(v) for k, v in res.items()}
        cell = lambda k: f"{med[k]:.1f}" if k in med else "-"  # noqa: E731
        print(f"| {name} | {cell('fwd_y')} | {cell('fwd_nol')} | {cell('dg_y')} | {cell('dg_c')} | {cell('wg_y')} | "
              f"{cell('wg_nol')} | {ok} |", flush=True)


if __name__ == "__main__":
    main()
