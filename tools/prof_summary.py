#!/usr/bin/env python
"""Summarise a rocprofv3 ``--kernel-trace --stats`` run into a markdown table (per-kernel
totals, share, calls, and per-step time).

    python tools/prof_summary.py gpurun_out/prof1/run_kernel_stats.csv --steps 5 > profiles/x.md
    python tools/prof_summary.py gpurun_out/prof1/run_results.db --steps 5   # rocpd SQLite output
    python tools/prof_summary.py run_results.db --marker sgd_flat_kernel --skip 3
        steady state only: the trace is cut into steps at each launch of the marker kernel (the
        fused optimizer ends every training step), the first --skip steps (and everything before
        them: model build, flat-buffer packing, warm-up) are dropped, and every per-step figure is
        over the remaining whole steps -- so one-off start-up launches (parameter packing copies)
        are not smeared over the steps.

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
    ap.add_argument("--marker", default=None, help="kernel (substring) launched once at the end of every step")
    ap.add_argument("--skip", type=int, default=1, help="with --marker: leading steps to drop")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    a = ap.parse_args()
    steps = a.steps
    if a.stats_csv.endswith(".db"):
        rows, steps = _rows_from_db(a.stats_csv, a.marker, a.skip, a.steps)
    else:
        rows = list(csv.DictReader(open(a.stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"## {a.title}\n")
    print(f"Total GPU kernel time: {tot / 1e6:.2f} ms over {steps} step(s) = **{tot / 1e6 / steps:.2f} ms/step**\n")
    print("| kernel | ms/step | share | calls/step | avg us |")
    print("|---|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: a.top]:
        t = float(r["TotalDurationNs"])
        print(f"| `{short(r['Name'])}` | {t / 1e6 / steps:.3f} | {100 * t / tot:.1f}% | "
              f"{int(r['Calls']) / steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} |")
    blits = [r for r in rows if "rocclr" in r["Name"] or "at::native" in r["Name"]]
    if blits:
        print("\nNon-native launches (runtime blits and ATen kernels) per step:\n")
        print("| kernel | calls/step | ms/step |\n|---|---:|---:|")
        for r in sorted(blits, key=lambda r: -int(r["Calls"])):
            print(f"| `{short(r['Name'])}` | {int(r['Calls']) / steps:.2f} | {float(r['TotalDurationNs']) / 1e6 / steps:.3f} |")


def _rows_from_db(path, marker, skip, steps):
    c = sqlite3.connect(path)
    q = "select name, start, end, stream, end - start from kernels"
    ks = list(c.execute(q))
    lo = min(k[1] for k in ks)
    hi = max(k[2] for k in ks)
    if marker:
        ends = sorted(k[2] for k in ks if marker in k[0])
        if len(ends) <= skip:
            raise SystemExit(f"only {len(ends)} '{marker}' launches; nothing left after --skip {skip}")
        lo, hi = ends[skip - 1] if skip > 0 else lo, ends[-1]
        steps = len(ends) - skip
        ks = [k for k in ks if k[1] >= lo and k[1] < hi]
        print(f"Steady state: {steps} step(s) between launch {skip} and launch {len(ends)} of `{marker}` "
              f"({(hi - lo) / 1e6 / steps:.2f} ms/step of wall time)\n")
    agg = {}
    for n, s, e, st, d in ks:
        t, k = agg.get(n, (0, 0))
        agg[n] = (t + d, k + 1)
    rows = [{"Name": n, "TotalDurationNs": str(t), "Calls": str(k), "AverageNs": str(t / max(k, 1))}
            for n, (t, k) in agg.items()]
    busy = sum(k[4] for k in ks)
    print(f"Kernel timeline span: {(hi - lo) / 1e6:.1f} ms; summed kernel time {busy / 1e6:.1f} ms "
          f"({100 * busy / max(hi - lo, 1):.0f}% of the span)\n")
    per = {}
    for n, s, e, st, d in ks:
        t, k = per.get(st, (0, 0))
        per[st] = (t + d, k + 1)
    if len(per) > 1:
        print("| stream | kernels/step | kernel ms/step |\n|---|---:|---:|")
        for st, (t, k) in sorted(per.items(), key=lambda x: -x[1][0]):
            print(f"| {st} | {k / steps:.1f} | {t / 1e6 / steps:.2f} |")
        print()
    return rows, steps


if __name__ == "__main__":
    main()
