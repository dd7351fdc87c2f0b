"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel family.

    python tools/pmc_summary.py gpurun_out/pmc1/run_counter_collection.csv [more.csv ...] --top 12

Each CSV row is one (dispatch, counter) pair; values are summed per kernel name over all
dispatches, and the derived ratios used in profiles/ are printed as a markdown table:
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x SIMDs per CU... as reported by the
counter, normalised by the kernel's own busy cycles), wait / issue-stall / active shares of wave
cycles, LDS bank-conflict cycles per LDS-active cycle, and HBM-side bytes (FETCH_SIZE /
WRITE_SIZE, KB) per dispatch.
"""
import argparse
import csv
from collections import defaultdict


def load(paths):
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for p in paths:
        with open(p, newline="") as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "?")
                name = name.replace("(anonymous namespace)::", "")
                if name.endswith(")") and "(" in name:
                    name = name[: name.rfind("(")]
                name = name.strip()
                acc[name][row["Counter_Name"]] += float(row["Counter_Value"])
                calls[name].add((p, row.get("Dispatch_Id", row.get("Correlation_Id"))))
    return acc, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    acc, calls = load(a.csv)
    order = sorted(acc, key=lambda k: -acc[k].get("SQ_BUSY_CYCLES", 0.0))[: a.top]
    print("| kernel | dispatches | MFMA busy / busy | WAIT_ANY | WAIT_INST_ANY | ACTIVE_INST | LDS conflict / LDS active "
          "| FETCH MB / call | WRITE MB / call |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in order:
        c = acc[k]
        waves_cyc = c.get("SQ_WAIT_ANY", 0) + c.get("SQ_WAIT_INST_ANY", 0) + c.get("SQ_ACTIVE_INST_ANY", 0)

        def pct(x, d):
            return f"{100.0 * x / d:.1f}%" if d else "-"

        n_sq = max(1, sum(1 for (p, _) in calls[k] if "pmc1" in p))
        n_f = max(1, sum(1 for (p, _) in calls[k] if "pmc2" in p))
        n_w = max(1, sum(1 for (p, _) in calls[k] if "pmc3" in p))
        fetch = f"{c['FETCH_SIZE'] / 1024.0 / n_f:.1f}" if "FETCH_SIZE" in c else "-"
        write = f"{c['WRITE_SIZE'] / 1024.0 / n_w:.1f}" if "WRITE_SIZE" in c else "-"
        print(f"| `{k[:60]}` | {n_sq} | {pct(c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0), c.get('SQ_BUSY_CYCLES', 0))} "
              f"| {pct(c.get('SQ_WAIT_ANY', 0), waves_cyc)} | {pct(c.get('SQ_WAIT_INST_ANY', 0), waves_cyc)} "
              f"| {pct(c.get('SQ_ACTIVE_INST_ANY', 0), waves_cyc)} "
              f"| {pct(c.get('SQ_LDS_BANK_CONFLICT', 0), c.get('SQ_ACTIVE_INST_LDS', 0))} | {fetch} | {write} |")


if __name__ == "__main__":
    main()
