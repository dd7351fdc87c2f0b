#!/usr/bin/env python
"""Run one GEMM shape repeatedly (for rocprofv3 --pmc counter collection).
    python tools/gemm_one.py --op nt --M 50432 --N 3072 --K 768 --iters 20"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="nt", choices=["nt", "nt256", "tn", "tn256", "blas", "blas_tn"])
    ap.add_argument("--M", type=int, default=50432)
    ap.add_argument("--N", type=int, default=3072)
    ap.add_argument("--K", type=int, default=768)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    BF = torch.bfloat16
    M, N, K = a.M, a.N, a.K
    A = (torch.rand(M, K, device="cuda") * 2 - 1).to(BF)
    B = (torch.rand(N, K, device="cuda") * 2 - 1).to(BF)
    C = torch.empty(M, N, dtype=BF, device="cuda")
    dY = (torch.rand(M, N, device="cuda") * 2 - 1).to(BF)
    dW = torch.zeros(N, K, dtype=torch.float32, device="cuda")
    st = stream_of(A)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(a.iters + 2):
        if it == 2:
            s.record()
        if a.op == "nt":
            _lib.call("mi_gemm_nt", ptr(A), ptr(B), ptr(C), ptr(None), ptr(None), M, N, K, K, K, N, 0, 0, st)
        elif a.op == "nt256":
            _lib.call("mi_gemm256_nt", ptr(A), ptr(B), ptr(C), ptr(None), ptr(None), 0, M, N, K, K, K, N, 0, 0, st)
        elif a.op == "tn256":
            _lib.call("mi_gemm256_tn", ptr(dY), ptr(A), ptr(dW), N, K, M, N, K, K, st)
        elif a.op == "blas_tn":
            torch.matmul(dY.t(), A)
        elif a.op == "tn":
            _lib.call("mi_gemm_tn", ptr(dY), ptr(A), ptr(dW), N, K, M, N, K, K, st)
        else:
            torch.matmul(A, B.t())
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    print(f"{a.op} M={M} N={N} K={K}: {ms:.3f} ms, {2.0 * M * N * K / ms / 1e9:.0f} TFLOP/s")


if __name__ == "__main__":
    main()
