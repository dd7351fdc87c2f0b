#!/usr/bin/env python
"""1x1 stride-1 conv weight gradients (ResNet bs256 shapes): the 128-tile implicit-GEMM TN kernel vs the
256x256 TN GEMM (mi_set_wgrad256), one process, interleaved rounds, medians.
    python tools/bench_wgrad256.py [--rounds 5] [--iters 10]"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

# (H, C = conv input channels, K = conv output channels)
SHAPES = [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024), (14, 1024, 256),
          (7, 512, 2048), (7, 2048, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    lib = _lib.load(True)
    CL, BF = torch.channels_last, torch.bfloat16
    print("| H | C | K | tn128 us | gemm256_tn us | TF/s (128 / 256) |")
    print("|---:|---:|---:|---:|---:|---:|")
    for (H, C, K) in SHAPES:
        Nb = a.batch
        x = torch.randn(Nb, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        dy = torch.randn(Nb, K, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        dw = torch.zeros(K, C, device="cuda")
        st = stream_of(x)

        def timed(t):
            lib.mi_set_wgrad256(t)
            _lib.call("mi_conv2d_wgrad", ptr(x), ptr(dy), ptr(dw), Nb, H, H, C, K, 1, 1, 1, 0, H, H, st)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                _lib.call("mi_conv2d_wgrad", ptr(x), ptr(dy), ptr(dw), Nb, H, H, C, K, 1, 1, 1, 0, H, H, st)
            e1.record()
            torch.cuda.synchronize()
            lib.mi_set_wgrad256(0)
            return e0.elapsed_time(e1) / a.iters * 1e3
        ts = {0: [], 1: []}
        for _ in range(a.rounds):
            for t in (0, 1):
                ts[t].append(timed(t))
        t0, t1 = statistics.median(ts[0]), statistics.median(ts[1])
        fl = 2.0 * Nb * H * H * C * K
        print(f"| {H} | {C} | {K} | {t0:.1f} | {t1:.1f} | {fl / t0 / 1e6:.0f} / {fl / t1 / 1e6:.0f} |")


if __name__ == "__main__":
    main()
