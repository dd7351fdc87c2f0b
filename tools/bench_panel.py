#!/usr/bin/env python
"""A/B of the 1x1 conv forward (+ BN statistics) on the persistent resident-weight panel kernel
(conv_panel.hip) vs the 128-tile nt_kernel, every ResNet-50 bs256 1x1 shape the panel takes, in ONE
process with interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  Reports us per call and the
achieved HBM bandwidth over the bytes the conv must move (input read once, output written once).

    python tools/bench_panel.py [--rounds 5] [--iters 20]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

BF, CL = torch.bfloat16, torch.channels_last

# forward: (C, H, K, stride, R, count per ResNet-50 step) at batch 256
SHAPES = [
    (64, 56, 64, 1, 1, 1), (64, 56, 256, 1, 1, 4), (256, 56, 64, 1, 1, 2), (256, 56, 128, 1, 1, 1),
    (128, 28, 512, 1, 1, 4), (512, 28, 128, 1, 1, 3), (256, 56, 512, 2, 1, 1), (256, 14, 1024, 1, 1, 6),
    (64, 56, 64, 1, 3, 3),
]
# data gradient with the step's epilogues: (C = dx channels, H, K = dy channels, R, epi, count)
DGRAD = [
    (256, 56, 64, 1, 5, 2), (64, 56, 256, 1, 4, 3), (256, 56, 128, 1, 5, 1), (512, 28, 128, 1, 5, 3),
    (128, 28, 512, 1, 4, 4), (1024, 14, 256, 1, 5, 5), (256, 14, 1024, 1, 4, 6), (64, 56, 64, 3, 4, 3),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    from mi355x_dp.ops._lib import ptr, stream_of
    lib = _lib.load(True)
    Nb = a.batch
    print("| conv | panel us | old us | speedup | panel TB/s | old TB/s | x count |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    tot_p = tot_o = 0.0
    def ab(run):
        def timed():
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / a.iters * 1e3
        tp, to = [], []
        for _ in range(a.rounds):
            lib.mi_set_panel(5)
            tp.append(timed())
            lib.mi_set_panel(0)
            to.append(timed())
        lib.mi_set_panel(5)
        return statistics.median(tp), statistics.median(to)

    for (C, H, K, s, R, cnt) in SHAPES:
        pad = R // 2
        P = (H + 2 * pad - R) // s + 1
        M = Nb * P * P
        x = torch.randn(Nb, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        w = (torch.randn(K, C, R, R, device="cuda") * 0.1).to(BF).contiguous(memory_format=CL)
        y = torch.empty(Nb, K, P, P, dtype=BF, device="cuda", memory_format=CL)
        slab = torch.empty(8192, 2, K, device="cuda")
        st = stream_of(x)

        def run():
            _lib.call("mi_conv2d_fwd", ptr(x), ptr(w), ptr(y), ptr(None), ptr(slab), Nb, H, H, C, K, R, R, s, pad, P,
                      P, 0, st)

        mp, mo = ab(run)
        routed = lib.mi_panel_stat_rows(M, K, C * R * R) > 0  # (mode 5: 3x3 included)
        byts = (Nb * H * H * C if s == 1 else M * C) * 2 + M * K * 2
        tot_p += mp * cnt
        tot_o += mo * cnt
        print(f"| fwd {C} {H} {K} s{s} {R}x{R} | {mp:.1f}{'' if routed else ' (not routed)'} | {mo:.1f} | "
              f"{mo / mp:.2f}x | {byts / mp / 1e6:.2f} | {byts / mo / 1e6:.2f} | {cnt} |")
        del x, w, y
    for (C, H, K, R, epi, cnt) in DGRAD:
        M = Nb * H * H
        dy = torch.randn(Nb, K, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        w = (torch.randn(K, C, R, R, device="cuda") * 0.1).to(BF).contiguous(memory_format=CL)
        wt = torch.empty(C, R, R, K, dtype=BF, device="cuda")
        st = stream_of(dy)
        _lib.call("mi_conv_wtrans", ptr(w), ptr(wt), K, R * R, C, st)
        dx = torch.randn(Nb, C, H, H, device="cuda").to(BF).contiguous(memory_format=CL)
        xin = torch.randn_like(dx)
        bits = torch.randint(0, 255, (M, C // 8), dtype=torch.uint8, device="cuda")
        mean = torch.zeros(C, device="cuda")
        slab = torch.empty(8192, 2, C, device="cuda")

        def run():
            _lib.call("mi_conv2d_dgrad_ex4", ptr(dy), ptr(wt), ptr(dx), Nb, H, H, C, K, R, R, 1, R // 2, H, H, epi,
                      ptr(None), ptr(xin), ptr(mean), 1, ptr(slab), 0, ptr(None), ptr(None), ptr(bits), st)

        mp, mo = ab(run)
        routed = lib.mi_panel_stat_rows2(M, C, K * R * R, 1) > 0
        byts = M * K * 2 + M * C * 2 * (3 if epi == 5 else 2) + M * C // 8
        tot_p += mp * cnt
        tot_o += mo * cnt
        print(f"| dgrad{epi} {C} {H} {K} {R}x{R} | {mp:.1f}{'' if routed else ' (not routed)'} | {mo:.1f} | "
              f"{mo / mp:.2f}x | {byts / mp / 1e6:.2f} | {byts / mo / 1e6:.2f} | {cnt} |")
        del dy, w, wt, dx, xin
    print(f"\nper ResNet-50 step (x count): panel {tot_p / 1e3:.3f} ms vs nt {tot_o / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
