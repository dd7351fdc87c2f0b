#!/usr/bin/env python
"""LayerNorm forward / backward timing on the ViT-B/16 batch-256 shape (M = 50432 rows, D = 768),
as achieved bandwidth.  MI355X_DP_LN_BWD16=0 selects the 8-byte full-wave-row backward kernel.

    python tools/bench_ln.py [--M 50432] [--D 768]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=50432)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from mi355x_dp.ops import transformer as T
    M, D = a.M, a.D
    BF = torch.bfloat16
    x = (torch.randn(M, D, device="cuda") * 2 + 0.5).to(BF)
    w = torch.randn(D, device="cuda") * 0.5 + 1
    b = torch.randn(D, device="cuda") * 0.1
    dy = torch.randn(M, D, device="cuda").to(BF)
    dres = torch.randn(M, D, device="cuda").to(BF)
    y, mean, rstd = T._ln_fwd(x, w, b, 1e-6)

    def run(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / a.iters * 1e3

    tf = run(lambda: T._ln_fwd(x, w, b, 1e-6))
    tb = run(lambda: T._ln_bwd(dy, x, w, b, mean, rstd, dres=dres))
    mb = M * D * 2 / 1e6
    print(f"LN16={os.environ.get('MI355X_DP_LN_BWD16', '1')} M={M} D={D}: fwd {tf:.1f} us ({2 * mb / tf:.2f} TB/s), "
          f"bwd {tb:.1f} us ({4 * mb / tb:.2f} TB/s)")


if __name__ == "__main__":
    main()
