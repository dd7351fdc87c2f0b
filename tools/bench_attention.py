#!/usr/bin/env python
"""Native attention kernels (csrc/kernels/attention.hip) on the ViT-B/16 shape (batch 256, 197
tokens, 12 heads x 64): forward, backward at 4 and 8 waves per workgroup (interleaved rounds in one
process), and torch SDPA for reference.  Random operands.

    python tools/bench_attention.py [--batch 256] [--rounds 5]
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
    B, T, H, Dh = a.batch, 197, 12, 64
    D = H * Dh
    qkv = (torch.randn(B * T, 3 * D, device="cuda") * 0.5).to(BF)
    o = torch.empty(B * T, D, dtype=BF, device="cuda")
    lse = torch.empty(B * H * T, device="cuda")
    do = (torch.randn(B * T, D, device="cuda") * 0.5).to(BF)
    dvec = torch.empty(B * H * T, device="cuda")
    dqkv = torch.empty_like(qkv)
    st = stream_of(qkv)
    scale = 1.0 / Dh ** 0.5

    def fwd():
        _lib.call("mi_attn_fwd", ptr(qkv), ptr(o), ptr(lse), B, T, H, scale, st)

    def bwd():
        _lib.call("mi_attn_bwd", ptr(qkv), ptr(o), ptr(do), ptr(lse), ptr(dvec), ptr(dqkv), B, T, H, scale, st)
    fwd()
    res = {"fwd": [], "fwd4": [], "bwd_fused": [], "bwd4": [], "bwd8": [], "fwd_rot": []}
    for _ in range(a.rounds):
        res["fwd"].append(timeit(fwd))                # default: 8 waves, online softmax, 2 key-tile pairs per chunk
        _lib.call("mi_set_att_fwd_waves", 4)          # the 4-wave single-pass forward (A/B)
        res["fwd4"].append(timeit(fwd))
        _lib.call("mi_set_att_fwd_waves", 8)
        res["bwd_fused"].append(timeit(bwd))       # default: the single-kernel backward
        _lib.call("mi_set_att_fused_bwd", 0)      # the dQ + dK/dV kernel pair (A/B)
        _lib.call("mi_set_att_waves", 4)
        res["bwd4"].append(timeit(bwd))
        _lib.call("mi_set_att_waves", 8)
        res["bwd8"].append(timeit(bwd))
        _lib.call("mi_set_att_fused_bwd", 1)
        _lib.call("mi_set_att_rotate", 1)         # the rotated tile deal (A/B; 4-wave forward only)
        _lib.call("mi_set_att_fwd_waves", 4)
        res["fwd_rot"].append(timeit(fwd))
        _lib.call("mi_set_att_fwd_waves", 8)
        _lib.call("mi_set_att_rotate", 0)
    # reference: the same layout through SDPA (time only)
    q, k, v = qkv.view(B, T, 3, H, Dh).permute(2, 0, 3, 1, 4).unbind(0)
    q, k, v = (t.contiguous().requires_grad_() for t in (q, k, v))

    def sdpa_fb():
        out = torch.nn.functional.scaled_dot_product_attention(q, k, v)
        out.backward(torch.ones_like(out))
    t_sdpa = statistics.median(timeit(sdpa_fb, 5) for _ in range(3))
    fl_f = 4.0 * B * H * T * T * Dh
    t = {k: statistics.median(v) for k, v in res.items()}
    print(f"| op | ms per layer | TF/s |\n|---|---:|---:|")
    print(f"| forward, 8 waves, online softmax (default) | {t['fwd']:.3f} | {fl_f / t['fwd'] / 1e9:.0f} |")
    print(f"| forward, 4 waves, single pass | {t['fwd4']:.3f} | {fl_f / t['fwd4'] / 1e9:.0f} |")
    print(f"| backward, one fused kernel (default) | {t['bwd_fused']:.3f} | {2.5 * fl_f / t['bwd_fused'] / 1e9:.0f} |")
    print(f"| backward, dQ + dK/dV kernels, 4 waves | {t['bwd4']:.3f} | {2.5 * fl_f / t['bwd4'] / 1e9:.0f} |")
    print(f"| backward, dQ + dK/dV kernels, 8 waves | {t['bwd8']:.3f} | {2.5 * fl_f / t['bwd8'] / 1e9:.0f} |")
    print(f"| torch SDPA fwd+bwd | {t_sdpa:.3f} | {3.5 * fl_f / t_sdpa / 1e9:.0f} |")
    print(f"| forward 4 waves, rotated tile deal | {t['fwd_rot']:.3f} | {fl_f / t['fwd_rot'] / 1e9:.0f} |")
    print(f"12 layers: fwd + bwd(fused) = {12 * (t['fwd'] + t['bwd_fused']):.2f} ms/step "
          f"(two kernels, 8 waves: {12 * (t['fwd'] + t['bwd8']):.2f})")

if __name__ == "__main__":
    main()
