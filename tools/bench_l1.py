#!/usr/bin/env python
"""Isolated timings of the ResNet-50 layer-1 convolutions (batch 256, 56x56: the 1x1s and the 3x3
halo tiles) with the fused epilogues the training step uses, as achieved HBM bandwidth over the bytes each one must move:
is a kernel at its memory roofline in isolation (then its in-model time is contention), or not?

    python tools/bench_l1.py [--iters 20] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mi355x_dp.ops import _lib  # noqa: E402
from mi355x_dp.ops import kernels  # noqa: E402,F401
from mi355x_dp.ops._lib import ptr  # noqa: E402

BF16, F32 = torch.bfloat16, torch.float32
CL = torch.channels_last


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
    Nb, H = a.batch, 56
    M = Nb * H * H

    def t(C):
        return torch.randn(Nb, C, H, H, device=dev).to(BF16).contiguous(memory_format=CL)

    x64, x256 = t(64), t(256)
    c256, acc256 = t(256), t(256)
    c64 = t(64)
    w_64_256 = (torch.randn(256, 64, device=dev) * 0.1).to(BF16).contiguous()    # fwd 64 -> 256: [K][C]
    w_256_64 = (torch.randn(64, 256, device=dev) * 0.1).to(BF16).contiguous()    # fwd 256 -> 64
    y256 = torch.empty(Nb, 256, H, H, dtype=BF16, device=dev, memory_format=CL)
    y64 = torch.empty(Nb, 64, H, H, dtype=BF16, device=dev, memory_format=CL)
    mean256, mean64 = torch.zeros(256, device=dev), torch.zeros(64, device=dev)
    bits256 = torch.randint(0, 255, (Nb, H, H, 32), dtype=torch.uint8, device=dev)
    bits64 = torch.randint(0, 255, (Nb, H, H, 8), dtype=torch.uint8, device=dev)

    def slab_f(C, K):
        rows = lib.mi_conv_stat_rows_g(Nb, H, H, C, K, 1, 1, 1, 0, H, H)
        return torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, K), dtype=F32, device=dev)

    def slab_d(C, K):
        rows = lib.mi_dgrad_stat_rows(Nb, H, H, C, H, H, 1, K, 1)
        return torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, C), dtype=F32, device=dev)

    sf256, sf64 = slab_f(64, 256), slab_f(256, 64)
    sd256, sd64 = slab_d(256, 64), slab_d(64, 256)
    w3 = (torch.randn(64, 9 * 64, device=dev) * 0.05).to(BF16).contiguous()     # 3x3 64 -> 64: [K][R][S][C]
    sf3 = torch.empty((lib.mi_conv_stat_rows_g(Nb, H, H, 64, 64, 3, 3, 1, 1, H, H) + lib.mi_bn_slab_extra_rows(), 2,
                       64), dtype=F32, device=dev)
    sd3 = torch.empty((lib.mi_dgrad_stat_rows(Nb, H, H, 64, H, H, 1, 64, 9) + lib.mi_bn_slab_extra_rows(), 2, 64),
                      dtype=F32, device=dev)
    y64b = torch.empty_like(y64)
    MB = M * 2 / 1e6  # MB per channel-plane... bytes of one bf16 channel over all pixels

    cases = [
        # name, fn, bytes moved (MB)
        ("fwd 64->256 + stats", lambda: _lib.call(
            "mi_conv2d_fwd", ptr(x64), ptr(w_64_256), ptr(y256), ptr(None), ptr(sf256), Nb, H, H, 64, 256, 1, 1, 1, 0,
            H, H, 0, st), (64 + 256) * MB),
        ("fwd 256->64 + stats", lambda: _lib.call(
            "mi_conv2d_fwd", ptr(x256), ptr(w_256_64), ptr(y64), ptr(None), ptr(sf64), Nb, H, H, 256, 64, 1, 1, 1, 0,
            H, H, 0, st), (256 + 64) * MB),
        # data gradient of a 256 -> 64 conv (dy 64 ch -> dx 256 ch) with epi 5 (accumulate, mask bits, stats)
        ("dgrad 64->256 epi5 bits", lambda: _lib.call(
            "mi_conv2d_dgrad_ex4", ptr(c64), ptr(w_64_256), ptr(acc256), Nb, H, H, 256, 64, 1, 1, 1, 0, H, H, 5,
            ptr(None), ptr(c256), ptr(mean256), 1, ptr(sd256), 0, ptr(None), ptr(None), ptr(bits256), st),
         (64 + 256 + 256 + 256 + 256 / 16) * MB),
        # data gradient of a 64 -> 256 conv (dy 256 ch -> dx 64 ch) with epi 4 (mask bits, stats)
        ("dgrad 256->64 epi4 bits", lambda: _lib.call(
            "mi_conv2d_dgrad_ex4", ptr(x256), ptr(w_256_64), ptr(y64), Nb, H, H, 64, 256, 1, 1, 1, 0, H, H, 4,
            ptr(None), ptr(c64), ptr(mean64), 1, ptr(sd64), 0, ptr(None), ptr(None), ptr(bits64), st),
         (256 + 64 + 64 + 64 / 16) * MB),
        # 3x3 / stride 1 halo tiles (conv2 of each layer-1 block): forward + stats, data gradient
        # with epi 4 (mask bits, BN-backward statistics) and plain (the epilogue's share)
        ("fwd 3x3 64->64 + stats (halo)", lambda: _lib.call(
            "mi_conv2d_fwd", ptr(x64), ptr(w3), ptr(y64b), ptr(None), ptr(sf3), Nb, H, H, 64, 64, 3, 3, 1, 1,
            H, H, 0, st), (64 + 64) * MB),
        ("dgrad 3x3 64->64 epi4 bits (halo)", lambda: _lib.call(
            "mi_conv2d_dgrad_ex4", ptr(c64), ptr(w3), ptr(y64b), Nb, H, H, 64, 64, 3, 3, 1, 1, H, H, 4,
            ptr(None), ptr(x64), ptr(mean64), 1, ptr(sd3), 0, ptr(None), ptr(None), ptr(bits64), st),
         (64 + 64 + 64 + 64 / 16) * MB),
        ("dgrad 3x3 64->64 plain (halo)", lambda: _lib.call(
            "mi_conv2d_dgrad_ex4", ptr(c64), ptr(w3), ptr(y64b), Nb, H, H, 64, 64, 3, 3, 1, 1, H, H, 0,
            ptr(None), ptr(None), ptr(None), 0, ptr(None), 0, ptr(None), ptr(None), ptr(None), st),
         (64 + 64) * MB),
    ]
    res = {n: [] for n, _, _ in cases}
    for _ in range(a.rounds):
        for n, fn, _ in cases:
            res[n].append(timed(fn, a.iters))
    print("| kernel | us | MB moved | TB/s |\n|---|---:|---:|---:|")
    for n, _, mb in cases:
        us = statistics.median(res[n])
        print(f"| {n} | {us:.1f} | {mb:.0f} | {mb / us:.2f} |")


if __name__ == "__main__":
    main()
