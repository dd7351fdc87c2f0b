#!/usr/bin/env python
"""Probe: do external events recorded inside a captured HIP graph let another stream start work
while the rest of the graph still runs?  (Design check for per-bucket collectives launched behind
a graphed backward: parallel/step_graph.py.)

The graph is [A: long work] ev.record() [B: long work].  After replay() the host makes a side
stream wait on ev and runs a tiny kernel there.  If the event node fires mid-graph, the side
kernel ends long before the graph does -- but not before A (the
wait must not be a no-op either).  Prints one JSON line."""
import json
import torch


def main():
    dev = torch.device("cuda:0")
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    y = torch.empty_like(x)
    s = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)
    ev = torch.cuda.Event(external=True)
    flag = torch.zeros(1, device=dev)

    def work(n):
        for _ in range(n):
            torch.matmul(x, x, out=y)

    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        work(2)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        work(20)
        ev.record()
        work(60)
    torch.cuda.synchronize()
    res = {}
    for it in range(3):
        t0 = torch.cuda.Event(enable_timing=True)
        t_side = torch.cuda.Event(enable_timing=True)
        t_end = torch.cuda.Event(enable_timing=True)
        main = torch.cuda.current_stream()
        t0.record(main)
        g.replay()
        t_end.record(main)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            flag.add_(1)
            t_side.record(side)
        torch.cuda.synchronize()
        res[it] = {"side_done_ms": t0.elapsed_time(t_side), "graph_done_ms": t0.elapsed_time(t_end)}
    ok = all(0.15 * r["graph_done_ms"] < r["side_done_ms"] < 0.6 * r["graph_done_ms"] for r in res.values())
    print(json.dumps({"probe": "graph_external_event", "overlap": ok, "runs": res, "flag": float(flag.item())}))


if __name__ == "__main__":
    main()
