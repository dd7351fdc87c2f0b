#!/usr/bin/env python
"""Host run-ahead of a training step from a rocprofv3 --hip-trace --kernel-trace rocpd database: for one
steady-state step (cut at the marker kernel), every synchronising HIP call (host blocked until the GPU
caught up) and, per kernel of the default stream, the lead = kernel start - end of its launch call (how
far ahead the host was; ~0 = the GPU waited for the host).
    python tools/host_lead.py run_results.db [--marker sgd_flat_kernel] [--step 5]"""
import argparse
import sqlite3

SYNC = ("hipMemcpyWithStream", "hipMemcpy", "hipDeviceSynchronize", "hipStreamSynchronize", "hipEventSynchronize",
        "hipMemcpyDtoH", "hipMemcpyHtoD", "hipMemset")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="sgd_flat_kernel")
    ap.add_argument("--step", type=int, default=5)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    kcols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    rcols = [r[1] for r in c.execute("pragma table_info(regions)")]
    print("kernels columns:", kcols)
    corr = next((x for x in ("corr_id", "correlation_id") if x in kcols), None)
    ks = list(c.execute(f"select name, start, end, stream{', ' + corr if corr else ''} from kernels order by start"))
    marks = [k for k in ks if a.marker in k[0]]
    t0, t1 = marks[a.step - 1][2], marks[a.step][2]  # from the end of one optimizer step to the next
    print(f"step {a.step}: GPU window {(t1 - t0) / 1e3:.1f} us")
    api = list(c.execute("select name, start, end, corr_id from regions where start >= ? and start < ? order by start",
                         (t0 - 30_000_000, t1)))
    print("\nsynchronising calls issued in the window (or up to 30 ms before it), us from the window start:")
    for n, s, e, _ in api:
        if n in SYNC:
            print(f"  {n:24s} at {(s - t0) / 1e3:9.1f}  blocked {(e - s) / 1e3:8.1f}")
    if not corr:
        return
    lrows = list(c.execute("select name, start, end, corr_id, id from regions where name like '%Launch%' "
                           "and start >= ? and start < ?", (t0 - 30_000_000, t1)))
    print("launch regions in range:", len(lrows), "sample:", lrows[:3])
    print("kernel sample:", [k for k in ks if t0 <= k[1] < t1][:3])
    # launches issued vs kernels started (all streams) at each point of the GPU window: their difference
    # is how many kernels the host was ahead (~0: the GPU waited for the host)
    import bisect
    lend = sorted(r[0] for r in c.execute("select end from regions where name like '%Launch%'"))
    kst = sorted(k[1] for k in ks)
    print("| GPU time (us) | launched | started | lead (kernels) |\n|---:|---:|---:|---:|")
    tt = t0
    while tt < t1:
        L, K = bisect.bisect_right(lend, tt), bisect.bisect_right(kst, tt)
        print(f"| {(tt - t0) / 1e3:.0f} | {L} | {K} | {L - K} |")
        tt += 250_000


if __name__ == "__main__":
    main()
