#!/usr/bin/env python
"""Run one conv kernel repeatedly (for rocprofv3 --pmc counter collection).
    python tools/conv_probe.py --kind fwd --N 256 --C 128 --H 28 --K 128 --R 3 --s 1 --iters 20"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

ap = argparse.ArgumentParser()
for k, v in dict(N=256, C=128, H=28, K=128, R=3, s=1, iters=20, stages=1).items():
    ap.add_argument(f"--{k}", type=int, default=v)
ap.add_argument("--kind", default="fwd")
a = ap.parse_args()
from mi355x_dp.ops import _lib, kernels  # noqa
from mi355x_dp.ops._lib import ptr, stream_of
_lib.load().mi_set_glds(1); _lib.load().mi_set_nt_stages(a.stages)
p = a.R // 2
P = (a.H + 2 * p - a.R) // a.s + 1
CL, BF = torch.channels_last, torch.bfloat16
x = torch.randn(a.N, a.C, a.H, a.H, device="cuda").to(BF).contiguous(memory_format=CL)
w = (torch.randn(a.K, a.C, a.R, a.R, device="cuda") * 0.05).to(BF).contiguous(memory_format=CL)
dy = torch.randn(a.N, a.K, P, P, device="cuda").to(BF).contiguous(memory_format=CL)
y = torch.empty(a.N, a.K, P, P, dtype=BF, device="cuda", memory_format=CL)
wt = torch.empty(a.C, a.R, a.R, a.K, dtype=BF, device="cuda")
dx = torch.empty_like(x)
dw = torch.zeros(a.K, a.R, a.R, a.C, device="cuda")
st = stream_of(x)
_lib.call("mi_conv_wtrans", ptr(w), ptr(wt), a.K, a.R * a.R, a.C, st)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(a.iters + 1):
    if it == 1:
        s.record()
    if a.kind == "fwd":
        _lib.call("mi_conv2d_fwd", ptr(x), ptr(w), ptr(y), ptr(None), ptr(None), a.N, a.H, a.H, a.C, a.K, a.R, a.R,
                  a.s, p, P, P, 0, st)
    elif a.kind == "dgrad":
        _lib.call("mi_conv2d_dgrad", ptr(dy), ptr(wt), ptr(dx), a.N, a.H, a.H, a.C, a.K, a.R, a.R, a.s, p, P, P, st)
    else:
        _lib.call("mi_conv2d_wgrad", ptr(x), ptr(dy), ptr(dw), a.N, a.H, a.H, a.C, a.K, a.R, a.R, a.s, p, P, P, st)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / a.iters
fl = 2.0 * a.N * P * P * a.K * a.C * a.R * a.R
print(f"{a.kind} N{a.N} C{a.C} H{a.H} K{a.K} R{a.R} s{a.s}: {ms:.3f} ms  {fl / ms / 1e9:.0f} TFLOP/s")
