#!/usr/bin/env python
"""For every non-native launch (runtime blit / ATen kernel) in ONE steady-state step of a rocprofv3
rocpd database, print the kernels launched just before and after it on the same stream -- where
in the step each stray launch comes from.

    python tools/prof_neighbors.py run_results.db --marker sgd_flat_kernel --step 5
"""
import argparse
import re
import sqlite3


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return n.split("(")[0][:70] if "<" not in n.split("(")[0] else n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="sgd_flat_kernel")
    ap.add_argument("--step", type=int, default=5)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    ks = list(c.execute("select name, start, end, stream from kernels order by start"))
    ends = [k[2] for k in ks if a.marker in k[0]]
    lo, hi = ends[a.step - 1], ends[a.step]
    step = [k for k in ks if lo <= k[1] < hi]
    for i, k in enumerate(step):
        if "at::native" in k[0] or "rocclr" in k[0]:
            same = [j for j in range(len(step)) if step[j][3] == k[3]]
            pos = same.index(i)
            prev = step[same[pos - 1]][0] if pos > 0 else "-"
            nxt = step[same[pos + 1]][0] if pos + 1 < len(same) else "-"
            print(f"{(k[1] - lo) / 1e3:9.1f} us  {short(k[0])}\n    after  {short(prev)}\n    before {short(nxt)}")


if __name__ == "__main__":
    main()
