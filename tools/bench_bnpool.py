#!/usr/bin/env python
"""The stem's BN + ReLU + 3x3/2 max-pool backward (mi_bnpool_bwd: statistics pass, finalize, apply) at the
ResNet-50 batch-256 shape, median of rounds (random inputs).
    python tools/bench_bnpool.py"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    lib = _lib.load(True)
    CL, BF, F32 = torch.channels_last, torch.bfloat16, torch.float32
    N, P, K, P2 = 256, 112, 64, 56
    c = torch.randn(N, K, P, P, device="cuda").to(BF).contiguous(memory_format=CL)
    dy = torch.randn(N, K, P2, P2, device="cuda").to(BF).contiguous(memory_format=CL)
    idx = torch.randint(0, 9, (N, P2, P2, K), dtype=torch.uint8, device="cuda")
    scale, shift = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.1
    gamma, mean, invstd = torch.ones(K, device="cuda"), torch.zeros(K, device="cuda"), torch.ones(K, device="cuda")
    gw, gb = torch.zeros(K, device="cuda"), torch.zeros(K, device="cuda")
    rows = max(lib.mi_bnpool_partial_rows(N * P * P, K), lib.mi_bnpool_partial_rows(N * P2 * P2, K))
    part = torch.empty((rows + lib.mi_bn_slab_extra_rows(), 2, K), dtype=F32, device="cuda")
    coef = torch.empty((3, K), dtype=F32, device="cuda")
    dc = torch.empty_like(c)
    st = stream_of(c)

    def once():
        _lib.call("mi_bnpool_bwd", ptr(dy), ptr(idx), ptr(c), ptr(dc), N, P, P, K, P2, P2, 3, 2, 1, ptr(scale),
                  ptr(shift), ptr(gamma), ptr(mean), ptr(invstd), ptr(gw), ptr(gb), ptr(coef), ptr(part), st)
    once()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            once()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10 * 1e3)
    print(f"bnpool_bwd: {statistics.median(ts):.1f} us (stats + finalize + apply)")


if __name__ == "__main__":
    main()
