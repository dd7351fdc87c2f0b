#!/usr/bin/env python
"""Per-launch-shape kernel time from a rocprofv3 rocpd database: dispatches grouped by (kernel,
grid size), steady-state steps only (cut at the marker kernel, as prof_summary.py), so a kernel
family's time can be attributed to the network layers that launch it (MI355X_DP_TRACE_GEMM=1
prints each GEMM / conv dispatch's geometry and block count on stderr).

    python tools/prof_by_grid.py run_results.db --marker sgd_flat_kernel --skip 3 [--match nt_kernel]
"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="sgd_flat_kernel")
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=60)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    gx = next((k for k in ("grid_size_x", "grid_x", "grid_size") if k in cols), None)
    gy = "grid_size_y" if "grid_size_y" in cols else None
    gz = "grid_size_z" if "grid_size_z" in cols else None
    wx = next((k for k in ("workgroup_size_x", "workgroup_x", "workgroup_size") if k in cols), None)
    sel = ", ".join(x for x in (gx, gy, gz, wx) if x)
    rows = list(c.execute(f"select name, start, end, stream, {sel} from kernels"))
    ends = sorted(r[2] for r in rows if a.marker in r[0])
    lo, hi = ends[a.skip - 1], ends[-1]
    steps = len(ends) - a.skip
    agg = {}
    for r in rows:
        if not (lo <= r[1] < hi) or a.match not in r[0]:
            continue
        name = re.sub(r"\(anonymous namespace\)::", "", r[0])
        name = name.split("(")[0] if "<" not in name.split("(")[0] else name[: name.index(">") + 1]
        grid = tuple(r[4:4 + len(sel.split(","))])
        t, k = agg.get((name, grid, r[3]), (0, 0))
        agg[(name, grid, r[3])] = (t + r[2] - r[1], k + 1)
    print(f"columns: {sel}; {steps} steady-state steps\n")
    print("| kernel | grid (x, y, z, wg) | stream | calls/step | us/call | ms/step |\n|---|---|---|---:|---:|---:|")
    for (n, g, st), (t, k) in sorted(agg.items(), key=lambda x: -x[1][0])[: a.top]:
        print(f"| `{n[:60]}` | {g} | {st} | {k / steps:.1f} | {t / k / 1e3:.1f} | {t / steps / 1e6:.3f} |")


if __name__ == "__main__":
    main()
