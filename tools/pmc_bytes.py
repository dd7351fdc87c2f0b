#!/usr/bin/env python
"""HBM-side traffic of a training step from rocprofv3 --pmc runs: FETCH_SIZE and WRITE_SIZE (KB per
dispatch, two separate counter runs -- together they exceed the 4 TCC counters of one pass) summed
per kernel family and divided by the number of optimizer steps (dispatches of --marker), then
compared with the step time.

    python tools/pmc_bytes.py --fetch F.csv --write W.csv --ms-per-step 20.5 [--top 30]
"""
import argparse
import csv
from collections import defaultdict


def load(path, counter):
    per = defaultdict(float)
    calls = defaultdict(set)
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row.get("Kernel_Name", "?").replace("(anonymous namespace)::", "")
            if name.endswith(")") and "(" in name:
                name = name[: name.rfind("(")]
            name = name.strip()[:80]
            per[name] += float(row["Counter_Value"])
            calls[name].add(row.get("Dispatch_Id", row.get("Correlation_Id")))
    return per, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--marker", default="sgd_flat_kernel")
    ap.add_argument("--ms-per-step", type=float, required=True)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    fet, fcalls = load(a.fetch, "FETCH_SIZE")
    wri, wcalls = load(a.write, "WRITE_SIZE")
    steps_f = max(1, len(fcalls.get(a.marker, ())))
    steps_w = max(1, len(wcalls.get(a.marker, ())))
    names = set(fet) | set(wri)
    rows = []
    for n in names:
        f = fet.get(n, 0.0) / steps_f / 1e6  # KB -> GB per step
        w = wri.get(n, 0.0) / steps_w / 1e6
        rows.append((f + w, f, w, len(fcalls.get(n, ())) / steps_f, n))
    rows.sort(reverse=True)
    tf = sum(r[1] for r in rows)
    tw = sum(r[2] for r in rows)
    print(f"steps counted: fetch {steps_f}, write {steps_w}")
    print(f"**HBM traffic per step: {tf:.2f} GB read + {tw:.2f} GB written = {tf + tw:.2f} GB;"
          f" over {a.ms_per_step} ms/step = {(tf + tw) / a.ms_per_step:.2f} TB/s average**\n")
    print("| kernel | calls/step | read GB/step | write GB/step |\n|---|---:|---:|---:|")
    for tot, f, w, c, n in rows[: a.top]:
        print(f"| `{n}` | {c:.1f} | {f:.3f} | {w:.3f} |")


if __name__ == "__main__":
    main()
