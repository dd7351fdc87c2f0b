#!/usr/bin/env python
"""The native 256x256 NT GEMMs of one ViT-B/16 encoder layer (batch 256: M = 50,432 tokens) timed
exactly as ops/transformer.py issues them -- qkv (+bias), proj (+bias, +residual), fc1 (+bias,
GELU, pre-activation aux out), fc2 (+bias, +residual), fc2 data gradient (GELU' from the aux) --
against the same shapes with no epilogue, each in two cache states: "hot" (the same operands
every call, as a microbenchmark loop sees them) and "cold" (a rotation over 6 operand sets, 1.9 GB,
past the 256 MB Infinity Cache, as inside the model).  Interleaved rounds, medians.

    python tools/bench_vit_layer_gemms.py [--batch 256] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

BF = torch.bfloat16
EPI_NONE, EPI_GELU, EPI_GELU_BWD, EPI_RESIDUAL = 0, 1, 2, 3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--sets", type=int, default=6)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    _lib.load(True)
    M = a.batch * 197
    D, F = 768, 3072
    # (name, N, K, epi, bias)
    cases = [("qkv", 3 * D, D, EPI_NONE, True), ("proj", D, D, EPI_RESIDUAL, True), ("fc1", F, D, EPI_GELU, True),
             ("fc2", D, F, EPI_RESIDUAL, True), ("fc2 dgrad", F, D, EPI_GELU_BWD, False)]
    g = torch.Generator(device="cuda").manual_seed(0)

    def rnd(*shape):
        return (torch.rand(*shape, device="cuda", generator=g) * 2 - 1).to(BF)

    print("| GEMM | M N K | epi | hot: plain ms | hot: fused ms | cold: plain ms | cold: fused ms | cold fused TF/s |")
    print("|---|---|---|---:|---:|---:|---:|---:|")
    for name, N, K, epi, has_bias in cases:
        sets = []
        for _ in range(a.sets):
            A, W = rnd(M, K), rnd(N, K)
            out = torch.empty(M, N, dtype=BF, device="cuda")
            aux = rnd(M, N) if epi in (EPI_GELU_BWD, EPI_RESIDUAL) else (
                torch.empty(M, N, dtype=BF, device="cuda") if epi == EPI_GELU else None)
            bias = torch.rand(N, device="cuda", generator=g) if has_bias else None
            sets.append((A, W, out, aux, bias))

        def call(s, fused):
            A, W, out, aux, bias = s
            e = epi if fused else EPI_NONE
            _lib.call("mi_gemm_nt_epi", ptr(A), ptr(W), ptr(out), ptr(bias if fused else None),
                      ptr(aux if e else None), e, M, N, K, K, K, N, stream_of(A))

        def timed(fused, cold, iters=12):
            for i in range(2):
                call(sets[i % len(sets)], fused)
            torch.cuda.synchronize()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s0.record()
            for i in range(iters):
                call(sets[i % len(sets)] if cold else sets[0], fused)
            s1.record()
            torch.cuda.synchronize()
            return s0.elapsed_time(s1) / iters

        res = {k: [] for k in ("hp", "hf", "cp", "cf")}
        for _ in range(a.rounds):
            res["hp"].append(timed(False, False))
            res["hf"].append(timed(True, False))
            res["cp"].append(timed(False, True))
            res["cf"].append(timed(True, True))
        med = {k: statistics.median(v) for k, v in res.items()}
        tf = 2.0 * M * N * K / med["cf"] / 1e9
        print(f"| {name} | {M} {N} {K} | {epi} | {med['hp']:.3f} | {med['hf']:.3f} | {med['cp']:.3f} | {med['cf']:.3f} "
              f"| {tf:.0f} |", flush=True)
        del sets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
