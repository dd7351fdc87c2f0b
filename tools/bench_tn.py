#!/usr/bin/env python
"""TN (weight-gradient) GEMM microbenchmark: C[M][N] += A[K][M]^T B[K][N] on the 128-tile split-K
kernel (mi_gemm_tn / mi_gemm_tn_bias, deterministic slabs) vs the deep-pipelined 256x256 kernel
(mi_gemm256_tn), on the ViT-B/16 Linear weight-gradient shapes and the ResNet-50 1x1-conv ones.

    python tools/bench_tn.py [--iters 10]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

SHAPES = [  # (name, M, N, K)
    ("vit qkv", 2304, 768, 50432), ("vit proj", 768, 768, 50432), ("vit fc1", 3072, 768, 50432),
    ("vit fc2", 768, 3072, 50432),
    ("rn50 l1 64->256", 256, 64, 802816), ("rn50 l1 256->64", 64, 256, 802816),
    ("rn50 l2 128->512", 512, 128, 200704), ("rn50 l2 512->128", 128, 512, 200704),
    ("rn50 l3 256->1024", 1024, 256, 50176), ("rn50 l3 1024->256", 256, 1024, 50176),
    ("rn50 l4 512->2048", 2048, 512, 12544), ("rn50 l4 2048->512", 512, 2048, 12544),
]


def timeit(fn, iters):
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
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    print("| shape | M N K | tn128 TF (ms) | tn128+bias TF (ms) | gemm256_tn TF (ms) | max rel diff 256 vs 128 |")
    print("|---|---|---:|---:|---:|---:|")
    for name, M, N, K in SHAPES:
        A = (torch.randn(K, M, device="cuda") * 0.1).to(torch.bfloat16)
        B = (torch.randn(K, N, device="cuda") * 0.1).to(torch.bfloat16)
        C1 = torch.zeros(M, N, device="cuda")
        C2 = torch.zeros(M, N, device="cuda")
        cs = torch.zeros(M, device="cuda")
        st = stream_of(A)
        fl = 2.0 * M * N * K

        def t128():
            C1.zero_()
            _lib.call("mi_gemm_tn", ptr(A), ptr(B), ptr(C1), M, N, K, M, N, N, st)

        def t128b():
            C1.zero_()
            cs.zero_()
            _lib.call("mi_gemm_tn_bias", ptr(A), ptr(B), ptr(C1), ptr(cs), M, N, K, M, N, N, st)

        def t256():
            C2.zero_()
            _lib.call("mi_gemm256_tn", ptr(A), ptr(B), ptr(C2), M, N, K, M, N, N, st)
        r = []
        for f in (t128, t128b, t256):
            ms = timeit(f, a.iters)
            r.append(f"{fl / ms / 1e9:.0f} ({ms:.3f})")
        t128()
        t256()
        torch.cuda.synchronize()
        d = float((C1 - C2).abs().max() / C1.abs().max().clamp_min(1e-30))
        print(f"| {name} | {M} {N} {K} | {r[0]} | {r[1]} | {r[2]} | {d:.1e} |", flush=True)


if __name__ == "__main__":
    main()
