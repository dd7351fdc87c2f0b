#!/usr/bin/env python
"""Plain-GEMM microbenchmark: native NT (C = A·Bᵀ, bf16 out) and TN (C = Aᵀ·B, fp32 out)
MFMA kernels vs torch.matmul (hipBLASLt) bf16 on square and ViT-B/16 shapes.  Random
[-1,1) operands (MFMA clocks differ on zero data).

    python tools/bench_gemm.py [--batch 128]
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
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    T = a.batch * 197
    shapes = [("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192),
              ("vit qkv", T, 2304, 768), ("vit proj", T, 768, 768),
              ("vit fc1", T, 3072, 768), ("vit fc2", T, 768, 3072)]
    print("| shape | M N K | NT TF (ms) | hipBLASLt A·Bᵀ TF (ms) | TN wgrad-form TF (ms) | hipBLASLt Aᵀ·B TF (ms) |")
    print("|---|---|---:|---:|---:|---:|")
    for name, M, N, K in shapes:
        fl = 2.0 * M * N * K
        A = (torch.rand(M, K, device="cuda") * 2 - 1).to(BF)
        B = (torch.rand(N, K, device="cuda") * 2 - 1).to(BF)
        C = torch.empty(M, N, dtype=BF, device="cuda")
        st = stream_of(A)
        t_nt = timeit(lambda: _lib.call("mi_gemm_nt", ptr(A), ptr(B), ptr(C), ptr(None), ptr(None), M, N, K, K, K,
                                        N, 0, 0, st))
        t_bl = timeit(lambda: torch.matmul(A, B.t()))
        # TN (weight-gradient form): dW[N,K] = dYᵀ[N,M] · X[M,K], reduction over the long M
        dY = (torch.rand(M, N, device="cuda") * 2 - 1).to(BF)
        dW = torch.zeros(N, K, dtype=torch.float32, device="cuda")
        t_tn = timeit(lambda: _lib.call("mi_gemm_tn", ptr(dY), ptr(A), ptr(dW), N, K, M, N, K, K, st))
        t_bt = timeit(lambda: torch.matmul(dY.t(), A))
        print(f"| {name} | {M} {N} {K} | {fl / t_nt / 1e9:.0f} ({t_nt:.3f}) | {fl / t_bl / 1e9:.0f} ({t_bl:.3f}) | "
              f"{fl / t_tn / 1e9:.0f} ({t_tn:.3f}) | {fl / t_bt / 1e9:.0f} ({t_bt:.3f}) |", flush=True)


if __name__ == "__main__":
    main()
