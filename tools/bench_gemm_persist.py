#!/usr/bin/env python
"""A/B of the 256x256 NT GEMM kernels on the ViT-B/16 shapes (batch 256: M = 50,432 tokens), bf16
out, in one process with interleaved rounds (cdna_hip_programming.md §5.4 rule 24): gemm256.hip
(one tile per block, epilogue after the loop) vs gemm256p.hip (persistent, epilogue under the next
tile's first k-step) vs torch.matmul (hipBLASLt).  Random [-1, 1) operands.

    python tools/bench_gemm_persist.py [--batch 256] [--rounds 5]
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
    # forward (bias) and data-gradient (no bias) GEMMs of one encoder layer
    shapes = [("qkv fwd", T, 2304, 768, True), ("proj fwd", T, 768, 768, True), ("fc1 fwd", T, 3072, 768, True),
              ("fc2 fwd", T, 768, 3072, True), ("qkv dgrad", T, 768, 2304, False), ("proj dgrad", T, 768, 768, False),
              ("fc1 dgrad", T, 768, 3072, False), ("fc2 dgrad", T, 3072, 768, False), ("sq8192", 8192, 8192, 8192, False)]
    print("| shape | M N K | gemm256 TF (ms) | gemm256p TF (ms) | hipBLASLt TF (ms) | p / 256 |")
    print("|---|---|---:|---:|---:|---:|")
    for name, M, N, K, has_bias in shapes:
        fl = 2.0 * M * N * K
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(BF)
        B = (torch.rand(N, K, device="cuda") * 2 - 1).to(BF)
        bias = torch.randn(N, device="cuda") if has_bias else None
        bias16 = bias.to(BF) if has_bias else None
        C = torch.empty(M, N, dtype=BF, device="cuda")
        st = stream_of(A)

        def g256():
            _lib.call("mi_gemm256_nt", ptr(A), ptr(B), ptr(C), ptr(bias), ptr(None), 0, M, N, K, K, K, N, 0, 0, st)

        def blas():
            torch.nn.functional.linear(A, B, bias16)
        res = {"old": [], "p": [], "blas": []}
        for _ in range(a.rounds):
            _lib.call("mi_set_gemm_persist", 0)
            res["old"].append(timeit(g256))
            _lib.call("mi_set_gemm_persist", 1)
            res["p"].append(timeit(g256))
            res["blas"].append(timeit(blas))
        _lib.call("mi_set_gemm_persist", 0)
        t = {k: statistics.median(v) for k, v in res.items()}
        print(f"| {name} | {M} {N} {K} | {fl / t['old'] / 1e9:.0f} ({t['old']:.3f}) | {fl / t['p'] / 1e9:.0f} "
              f"({t['p']:.3f}) | {fl / t['blas'] / 1e9:.0f} ({t['blas']:.3f}) | {t['old'] / t['p']:.3f} |", flush=True)


if __name__ == "__main__":
    main()
