#!/usr/bin/env python
"""A/B of the folded BatchNorm backward (ops/resblock.py _Fold) against the materialised one on the
ResNet-50 bs256 shapes it takes, component by component, in ONE process with interleaved rounds:

  materialised: BN-backward finalize + apply (mi_bn_bwd_train_pre: writes dX), the consumer 1x1 conv's
                data gradient of dX (mi_conv2d_dgrad_ex4) and weight gradient (mi_conv2d_wgrad);
  folded:       finalize only (mi_bn_bwd_coef), mi_panel_dgrad_fbb over [dz | c], mi_conv2d_wgrad_fbb over
                [dz | x] (c^T x = W x^T x).

    python tools/bench_fold.py [--rounds 5] [--iters 10]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

BF, CL = torch.bfloat16, torch.channels_last
# (name, H, K = BN channels (dz / c), C = the consumer conv's input channels, dgrad epilogue, count per step)
# (the folded path takes expansions only, K > C: the layer-1 conv3s; raw/r6/bench_fold_ab.log has the
# K < C conv1 shapes measured with the earlier [dz | c] weight gradient, all slower folded)
SHAPES = [("l1 bn3 -> conv3", 56, 256, 64, 4, 3)]


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
    Nb = a.batch

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters * 1e3

    print("| BN -> consumer | apply us | dgrad us | wgrad us | materialised us | coef us | fbb dgrad us | "
          "fbb wgrad us | folded us | x count |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    tot_m = tot_f = 0.0
    for (name, H, K, C, epi, cnt) in SHAPES:
        M = Nb * H * H
        g = torch.Generator(device="cuda").manual_seed(1)
        dz = torch.randn(Nb, K, H, H, device="cuda", generator=g).to(BF).contiguous(memory_format=CL)
        c = torch.randn(Nb, K, H, H, device="cuda", generator=g).to(BF).contiguous(memory_format=CL)
        x = torch.relu(torch.randn(Nb, C, H, H, device="cuda", generator=g)).to(BF).contiguous(memory_format=CL)
        w = (torch.randn(K, C, 1, 1, device="cuda", generator=g) * 0.05).to(BF).contiguous(memory_format=CL)
        wt = torch.empty(C, 1, 1, K, dtype=BF, device="cuda")
        st = stream_of(dz)
        _lib.call("mi_conv_wtrans", ptr(w), ptr(wt), K, 1, C, st)
        gamma, mean, invstd = torch.ones(K, device="cuda"), torch.zeros(K, device="cuda"), torch.ones(K, device="cuda")
        gw, gb = torch.zeros(K, device="cuda"), torch.zeros(K, device="cuda")
        coef = torch.zeros(3, K, device="cuda")
        pre_rows = 256
        part = torch.zeros(pre_rows + lib.mi_bn_slab_extra_rows(), 2, K, device="cuda")
        dX = torch.empty_like(dz)
        out = torch.randn(Nb, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        xin = torch.randn_like(out)
        mn = torch.zeros(C, device="cuda")
        bits = torch.randint(0, 255, (M, C // 8), dtype=torch.uint8, device="cuda")
        rows = max(lib.mi_dgrad_stat_rows(Nb, H, H, C, H, H, 1, K, 1), lib.mi_panel_fbb_rows(M, C, K))
        slab = torch.empty(rows + lib.mi_bn_slab_extra_rows(), 2, C, device="cuda")
        dw = torch.zeros(K, 1, 1, C, device="cuda")
        ws = torch.zeros(lib.mi_conv2d_wgrad_fbb_ws_floats(K, C), device="cuda")

        def apply_():
            _lib.call("mi_bn_bwd_train_pre", ptr(dz), ptr(c), ptr(dX), ptr(None), M, K, ptr(gamma), ptr(mean),
                      ptr(invstd), ptr(gw), ptr(gb), ptr(coef), ptr(part), pre_rows, st)

        def dgrad_():
            _lib.call("mi_conv2d_dgrad_ex4", ptr(dX), ptr(wt), ptr(out), Nb, H, H, C, K, 1, 1, 1, 0, H, H, epi,
                      ptr(None), ptr(xin), ptr(mn), 1, ptr(slab), 0, ptr(None), ptr(None), ptr(bits), st)

        def wgrad_():
            _lib.call("mi_conv2d_wgrad", ptr(x), ptr(dX), ptr(dw), Nb, H, H, C, K, 1, 1, 1, 0, H, H, st)

        def coef_():
            _lib.call("mi_bn_bwd_coef", M, K, ptr(gamma), ptr(mean), ptr(invstd), ptr(gw), ptr(gb), ptr(coef),
                      ptr(part), pre_rows, st)

        def fdgrad_():
            _lib.call("mi_panel_dgrad_fbb", ptr(dz), ptr(c), ptr(coef), ptr(wt), ptr(out), Nb, H, H, C, K, epi,
                      ptr(None), ptr(xin), ptr(mn), 1, ptr(slab), 0, ptr(bits), ptr(None), st)

        def fwgrad_():
            _lib.call("mi_conv2d_wgrad_fbb", ptr(x), ptr(dz), ptr(w), ptr(coef), ptr(dw), ptr(ws), Nb, H, H, C, K, st)

        fns = [apply_, dgrad_, wgrad_, coef_, fdgrad_, fwgrad_]
        ts = [[] for _ in fns]
        for _ in range(a.rounds):
            for i, f in enumerate(fns):
                ts[i].append(timed(f))
        t = [statistics.median(v) for v in ts]
        mat, fold = t[0] + t[1] + t[2], t[3] + t[4] + t[5]
        tot_m += mat * cnt
        tot_f += fold * cnt
        print(f"| {name} ({K} ch @ {H}², C {C}) | {t[0]:.1f} | {t[1]:.1f} | {t[2]:.1f} | {mat:.1f} | {t[3]:.1f} | "
              f"{t[4]:.1f} | {t[5]:.1f} | {fold:.1f} | {cnt} |")
    print(f"\nper ResNet-50 step (x count): materialised {tot_m / 1e3:.3f} ms, folded {tot_f / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
