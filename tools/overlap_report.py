#!/usr/bin/env python
"""Comm/compute overlap from a rocprofv3 kernel trace (rocpd SQLite) of one bench.py rank.

Collective kernels (RCCL or the smddp IPC kernels) run on the backend's comm stream; the step's
forward/backward/optimizer kernels run on the compute stream.  For every traced step (delimited
by the input-pipeline `augment_kernel`) this prints each collective's start / end relative to the
step start, how much of it ran while a compute kernel was running (overlapped), and the exposed
tail: time from the end of the last backward kernel to the end of the last collective.

    python tools/overlap_report.py gpurun_out/ipc_overlap_r0/run_results.db [--steps 3]
"""
import argparse
import re
import sqlite3

COMM = re.compile(r"ipc_|nccl|rccl|Nccl|Rccl", re.I)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=int, default=3, help="last N steps to report")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = [(n, s, b, e) for n, s, b, e in c.execute("select name, stream, start, end from kernels order by start")]
    comm_streams = {s for n, s, b, e in rows if COMM.search(n)}
    starts = [b for n, s, b, e in rows if "augment_kernel" in n]
    print(f"comm stream(s): {sorted(comm_streams)}; traced steps: {len(starts)}\n")
    print("| step | collective | size | start ms | end ms | overlapped with compute | backward end ms | exposed tail ms |")
    print("|---:|---|---|---:|---:|---:|---:|---:|")
    for k in range(max(0, len(starts) - 1 - a.steps), len(starts) - 1):
        t0, t1 = starts[k], starts[k + 1]
        step = [r for r in rows if t0 <= r[2] < t1]
        comp = [(b, e) for n, s, b, e in step if s not in comm_streams]
        comm = [(n, b, e) for n, s, b, e in step if s in comm_streams and COMM.search(n)]
        sgd = [b for n, s, b, e in step if "sgd_flat" in n]
        bwd_end = max((e for b, e in comp if not sgd or b < sgd[0]), default=t0)
        for i, (n, b, e) in enumerate(comm):
            ov = sum(max(0, min(e, ce) - max(b, cb)) for cb, ce in comp)
            short = re.sub(r"\(anonymous namespace\)::", "", n).replace("void ", "")
            short = re.sub(r"\(.*", "", short)[:28]
            tail = ""
            if i == len(comm) - 1:
                tail = f"{max(0, e - bwd_end) / 1e6:.3f}"
            print(f"| {k} | {short} | #{i} | {(b - t0) / 1e6:.3f} | {(e - t0) / 1e6:.3f} | "
                  f"{100 * ov / max(e - b, 1):.0f}% | {(bwd_end - t0) / 1e6:.3f} | {tail} |")


if __name__ == "__main__":
    main()
