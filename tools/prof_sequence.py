#!/usr/bin/env python
"""Print ONE steady-state step of a rocprofv3 rocpd database as an ordered kernel list per stream:
start offset, duration, grid and name -- maps each launch of a summary row back to its layer.

    python tools/prof_sequence.py run_results.db --marker sgd_flat_kernel --step 5 > seq.txt
"""
import argparse
import re
import sqlite3


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    head = n.split("(")[0]
    return head[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="sgd_flat_kernel")
    ap.add_argument("--step", type=int, default=5)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    gx = "grid_size_x" if "grid_size_x" in cols else ("grid_x" if "grid_x" in cols else None)
    wx = "workgroup_size_x" if "workgroup_size_x" in cols else ("workgroup_x" if "workgroup_x" in cols else None)
    sel = "name, start, end, stream" + (f", {gx}" if gx else ", 0") + (f", {wx}" if wx else ", 0")
    ks = list(c.execute(f"select {sel} from kernels order by start"))
    ends = [k[2] for k in ks if a.marker in k[0]]
    lo, hi = ends[a.step - 1], ends[a.step]
    step = [k for k in ks if lo <= k[1] < hi]
    streams = sorted({k[3] for k in step}, key=str)
    for s in streams:
        print(f"## stream {s}")
        tot = 0.0
        for k in step:
            if k[3] != s:
                continue
            d = (k[2] - k[1]) / 1e3
            tot += d
            blocks = k[4] // k[5] if k[5] else k[4]
            print(f"{(k[1] - lo) / 1e3:9.1f} {d:8.1f} {blocks:8d} {short(k[0])}")
        print(f"# total {tot:.1f} us")


if __name__ == "__main__":
    main()
