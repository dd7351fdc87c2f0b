#!/usr/bin/env python
"""Summarise a rocprofv3 ``--kernel-trace --stats --output-format csv`` run into a
markdown table (per-kernel totals, share, calls, and per-step time).

    python tools/prof_summary.py gpurun_out/prof1/run_kernel_stats.csv --steps 5 > profiles/x.md
    python tools/prof_summary.py gpurun_out/prof1/run_results.db --steps 5   # rocpd SQLite output

With a ``.db`` input it also reports the wall span of the kernel timeline, the GPU busy
fraction over it, and per-stream kernel time (comm-stream overlap evidence).
"""
import sqlite3
import argparse
import csv
import re


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*", "", name) if "<" not in name.split("(")[0] else name.split("(")[0]
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats_csv")
    ap.add_argument("--steps", type=int, default=1, help="number of training steps covered by the trace")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    a = ap.parse_args()
    if a.stats_csv.endswith(".db"):
        rows = _rows_from_db(a.stats_csv)
    else:
        rows = list(csv.DictReader(open(a.stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"## {a.title}\n")
    print(f"Total GPU kernel time: {tot / 1e6:.2f} ms over {a.steps} step(s) = **{tot / 1e6 / a.steps:.2f} ms/step**\n")
    print("| kernel | ms/step | share | calls/step | avg us |")
    print("|---|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: a.top]:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {t / 1e6 / a.steps:.3f} | {100 * t / tot:.1f}% | "
              f"{int(r['Calls']) / a.steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} |")


def _rows_from_db(path):
    c = sqlite3.connect(path)
    rows = [{"Name": n, "TotalDurationNs": str(t), "Calls": str(k), "AverageNs": str(t / max(k, 1))}
            for n, t, k in c.execute("select name, sum(duration), count(*) from kernels group by name")]
    lo, hi, busy = c.execute("select min(start), max(end), sum(duration) from kernels").fetchone()
    print(f"Kernel timeline span: {(hi - lo) / 1e6:.1f} ms; summed kernel time {busy / 1e6:.1f} ms "
          f"({100 * busy / max(hi - lo, 1):.0f}% of the span)\n")
    streams = list(c.execute("select stream, count(*), sum(duration) from kernels group by stream"))
    if len(streams) > 1:
        print("| stream | kernels | kernel ms |\n|---|---:|---:|")
        for st, k, t in streams:
            print(f"| {st} | {k} | {t / 1e6:.1f} |")
        print()
    return rows


if __name__ == "__main__":
    main()
