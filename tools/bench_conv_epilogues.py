#!/usr/bin/env python
"""What the fused epilogues of the ResNet-50 training step cost on top of the plain convolutions:
every distinct conv (batch 256) timed (a) forward plain vs forward + BN-statistics epilogue
(mi_conv2d_fwd with a statistics slab), (b) data gradient plain vs + BatchNorm-backward epilogue
(epi 4: ReLU mask of the producing BN's output + its backward statistics) and vs + accumulate
(epi 3), interleaved rounds, medians.  Counterpart of bench_vit_layer_gemms.py for the convs.

    python tools/bench_conv_epilogues.py [--batch 256] [--rounds 3]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from bench_conv import conv_shapes, timeit  # noqa: E402

CL = torch.channels_last
BF = torch.bfloat16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    lib = _lib.load(True)
    tot = {"fwd": 0.0, "fwd_stats": 0.0, "dgrad": 0.0, "dgrad_bn": 0.0, "dgrad_acc": 0.0}
    print("| N C H K R s | count | fwd ms | fwd+stats ms | dgrad ms | dgrad+BN-bwd ms | dgrad+acc ms |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for (N, C, H, K, R, s, p, cnt) in conv_shapes("resnet50", a.batch, 224):
        if C % 64:
            continue  # the stem has its own kernels
        P = (H + 2 * p - R) // s + 1
        x = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(BF).contiguous(memory_format=CL)
        wt = torch.empty((C, R, R, K), dtype=BF, device="cuda")
        _lib.call("mi_conv_wtrans", ptr(w), ptr(wt), K, R * R, C, stream_of(w))
        dy = torch.randn(N, K, P, P, device="cuda").to(BF).contiguous(memory_format=CL)
        y = torch.empty(N, K, P, P, dtype=BF, device="cuda", memory_format=CL)
        dx = torch.empty(N, C, H, H, dtype=BF, device="cuda", memory_format=CL)
        yprev = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        cprev = torch.randn(N, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        mean = torch.zeros(C, device="cuda")
        rows_f = lib.mi_conv_stat_rows_g(N, H, H, C, K, R, R, s, p, P, P)
        slab_f = torch.empty((rows_f + lib.mi_bn_slab_extra_rows(), 2, K), device="cuda")
        rows_b = lib.mi_dgrad_stat_rows(N, H, H, C, P, P, s, K, R * R)
        slab_b = torch.empty((rows_b + lib.mi_bn_slab_extra_rows(), 2, C), device="cuda")
        st = stream_of(x)

        def fwd(stats):
            _lib.call("mi_conv2d_fwd", ptr(x), ptr(w), ptr(y), ptr(None), ptr(slab_f if stats else None), N, H, H, C,
                      K, R, R, s, p, P, P, 0, st)

        def dgrad(epi):
            aux = {0: None, 3: dx, 4: yprev}[epi]
            _lib.call("mi_conv2d_dgrad_ex2", ptr(dy), ptr(wt), ptr(dx), N, H, H, C, K, R, R, s, p, P, P, epi, ptr(aux),
                      ptr(cprev if epi == 4 else None), ptr(mean if epi == 4 else None), int(epi == 4),
                      ptr(slab_b if epi == 4 else None), 0, st)

        fns = {"fwd": lambda: fwd(False), "fwd_stats": lambda: fwd(True), "dgrad": lambda: dgrad(0),
               "dgrad_bn": lambda: dgrad(4), "dgrad_acc": lambda: dgrad(3)}
        res = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                res[k].append(timeit(f))
        med = {k: statistics.median(v) for k, v in res.items()}
        for k in tot:
            tot[k] += med[k] * cnt
        print(f"| {N} {C} {H} {K} {R} {s} | {cnt} | {med['fwd']:.3f} | {med['fwd_stats']:.3f} | {med['dgrad']:.3f} | "
              f"{med['dgrad_bn']:.3f} | {med['dgrad_acc']:.3f} |", flush=True)
        del x, w, wt, dy, y, dx, yprev, cprev, slab_f, slab_b
        torch.cuda.empty_cache()
    print(f"\n**per step-equivalent (x count):** fwd {tot['fwd']:.2f} ms, fwd+stats {tot['fwd_stats']:.2f} ms, "
          f"dgrad {tot['dgrad']:.2f} ms, dgrad+BN-bwd {tot['dgrad_bn']:.2f} ms, dgrad+acc {tot['dgrad_acc']:.2f} ms")


if __name__ == "__main__":
    main()
