#!/usr/bin/env python
"""A/B of the ViT-B/16 weight-gradient GEMMs (batch 256: K = 50,432 tokens), fp32 gradient
accumulated into an existing buffer plus the bias gradient, in one process with interleaved
rounds: the native split-K TN kernel with the fused column sums (mi_gemm_tn_bias) vs the library
GEMM (torch.addmm with out_dtype=float32 -> hipBLASLt, accumulating in place) + mi_colsum_bf16,
and the native 256x256 TN kernel (mi_gemm256_tn, fp32 atomics across its K splits) + mi_colsum_bf16.

    python tools/bench_vit_wgrad.py [--batch 256] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

BF = torch.bfloat16


def timeit(fn, iters=10):
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
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    _lib.load(True)
    T = a.batch * 197
    # (name, out features N, in features K): dW[N][K] = dY[T][N]^T X[T][K]
    shapes = [("qkv", 2304, 768), ("proj", 768, 768), ("fc1", 3072, 768), ("fc2", 768, 3072)]
    print("| shape | T N K | native TN+colsum ms (TF/s) | hipBLASLt addmm + colsum ms (TF/s) | "
          "gemm256_tn + colsum ms (TF/s) | gemm256_tn alone ms (TF/s) | max rel diff (TN, 256) |")
    print("|---|---|---:|---:|---:|---:|---:|")
    for name, N, K in shapes:
        g = torch.Generator(device="cuda").manual_seed(0)
        dy = (torch.rand(T, N, device="cuda", generator=g) * 2 - 1).to(BF)
        x = (torch.rand(T, K, device="cuda", generator=g) * 2 - 1).to(BF)
        gw1 = torch.zeros(N, K, device="cuda")
        gb1 = torch.zeros(N, device="cuda")
        gw2 = torch.zeros(N, K, device="cuda")
        gb2 = torch.zeros(N, device="cuda")
        gw3 = torch.zeros(N, K, device="cuda")
        gb3 = torch.zeros(N, device="cuda")

        def native():
            _lib.call("mi_gemm_tn_bias", ptr(dy), ptr(x), ptr(gw1), ptr(gb1), N, K, T, N, K, K, stream_of(dy))

        def library():
            torch.addmm(gw2, dy.t(), x, out_dtype=torch.float32, out=gw2)
            _lib.call("mi_colsum_bf16", ptr(dy), ptr(gb2), T, N, N, stream_of(dy))

        def g256():
            _lib.call("mi_gemm256_tn", ptr(dy), ptr(x), ptr(gw3), N, K, T, N, K, K, stream_of(dy))
            _lib.call("mi_colsum_bf16", ptr(dy), ptr(gb3), T, N, N, stream_of(dy))

        def g256_only():
            _lib.call("mi_gemm256_tn", ptr(dy), ptr(x), ptr(gw3), N, K, T, N, K, K, stream_of(dy))

        native(); library(); g256()
        torch.cuda.synchronize()
        diff = float((gw1 - gw2).abs().max() / gw2.abs().max())
        diff3 = float((gw3 - gw2).abs().max() / gw2.abs().max())
        tn, tl, t3, t4 = [], [], [], []
        for _ in range(a.rounds):
            tn.append(timeit(native))
            tl.append(timeit(library))
            t3.append(timeit(g256))
            t4.append(timeit(g256_only))
        mn, ml, m3, m4 = (statistics.median(v) for v in (tn, tl, t3, t4))
        fl = 2.0 * T * N * K
        print(f"| {name} | {T} {N} {K} | {mn:.3f} ({fl / mn / 1e9:.0f}) | {ml:.3f} ({fl / ml / 1e9:.0f}) | "
              f"{m3:.3f} ({fl / m3 / 1e9:.0f}) | {m4:.3f} ({fl / m4 / 1e9:.0f}) | {diff:.1e} / {diff3:.1e} |",
              flush=True)


if __name__ == "__main__":
    main()
