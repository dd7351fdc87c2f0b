#!/usr/bin/env python
"""Design probes for structural comm/compute overlap in a replayed backward graph (VERDICT r4
item 3).  Prints one JSON line per probe.

1. ``branches``: does a HIP graph with a forked branch (s -> s2 fork, join at the end) replay its
   branches concurrently?  Both branches are one-thread spin kernels (``torch.cuda._sleep``), so
   concurrency shows as replay time ~T instead of ~2T.
2. ``rccl_capture``: a torch ``nccl`` (RCCL) all-reduce captured in the middle of a graph at world
   1 (async_op + wait inside the capture): does it capture, replay, and overlap the work after it?
3. ``wait_value``: hipStreamWaitValue32 on a side stream released by a kernel on another stream:
   the side stream's work must start only after the flag store, and the host must not block.
4. ``launch_host``: host wall time of ``replay()`` for a graph of N small kernels (per-node cost).
"""
import ctypes
import json
import os
import time

import torch
import torch.distributed as dist


def _ms(a, b):
    return a.elapsed_time(b)


def probe_branches(cycles=2_000_000):
    dev = torch.device("cuda:0")
    s, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    # calibrate one spin
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(cycles)
    e1.record()
    torch.cuda.synchronize()
    t1 = _ms(e0, e1)
    g = torch.cuda.CUDAGraph()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=s):
        s2.wait_stream(s)
        torch.cuda._sleep(cycles)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cycles)
        s.wait_stream(s2)
    torch.cuda.synchronize()
    times = []
    for _ in range(3):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        times.append(_ms(e0, e1))
    return {"probe": "branches", "one_spin_ms": round(t1, 3), "replay_ms": [round(t, 3) for t in times],
            "concurrent": min(times) < 1.5 * t1}


def probe_rccl_capture():
    dev = torch.device("cuda:0")
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    y = torch.empty_like(x)
    t = torch.ones(8 << 20, device=dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        w = dist.all_reduce(t, async_op=True)
        w.wait()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    res = {"probe": "rccl_capture"}
    try:
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            for _ in range(10):
                torch.matmul(x, x, out=y)
            w = dist.all_reduce(t, async_op=True)
            for _ in range(30):
                torch.matmul(x, x, out=y)
            w.wait()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times = []
        for _ in range(3):
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            times.append(round(_ms(e0, e1), 3))
        res.update(captured=True, replay_ms=times, value=float(t[0].item()))
    except Exception as e:  # noqa: BLE001 -- a probe reports, never fails
        res.update(captured=False, error=repr(e)[:400])
    return res


def probe_wait_value(cycles=2_000_000):
    dev = torch.device("cuda:0")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamWaitValue32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint, ctypes.c_uint32]
    hip.hipStreamWaitValue32.restype = ctypes.c_int
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    prod, side = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    marker = torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    e0, e_side, e_prod = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record(torch.cuda.current_stream())
    prod.wait_stream(torch.cuda.current_stream())
    side.wait_stream(torch.cuda.current_stream())
    # producer enqueued FIRST: should the two streams share a hardware queue, the wait packet then
    # sits behind the producer instead of blocking it (no deadlock either way)
    with torch.cuda.stream(prod):
        torch.cuda._sleep(cycles)
        flag.fill_(1)
        e_prod.record(prod)
    h0 = time.perf_counter()
    rc = hip.hipStreamWaitValue32(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(flag.data_ptr()), 1, 0x0,
                                  0xFFFFFFFF)
    with torch.cuda.stream(side):
        marker.add_(1)
        e_side.record(side)
    host_ms = (time.perf_counter() - h0) * 1e3
    torch.cuda.synchronize()
    return {"probe": "wait_value", "rc": rc, "host_enqueue_ms": round(host_ms, 3),
            "producer_done_ms": round(_ms(e0, e_prod), 3), "side_done_ms": round(_ms(e0, e_side), 3),
            "ordered": _ms(e0, e_side) >= _ms(e0, e_prod) - 0.01, "marker": float(marker.item())}


def probe_launch_host(n=300):
    dev = torch.device("cuda:0")
    a = torch.zeros(1024, device=dev)
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            a.add_(1)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    hs = []
    for _ in range(5):
        h0 = time.perf_counter()
        g.replay()
        hs.append((time.perf_counter() - h0) * 1e3)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return {"probe": "launch_host", "nodes": n, "host_replay_ms": [round(h, 3) for h in hs],
            "gpu_replay_ms": round(_ms(e0, e1), 3)}


def main():
    for fn in (probe_branches, probe_launch_host, probe_wait_value, probe_rccl_capture):
        try:
            print(json.dumps(fn()), flush=True)
        except Exception as e:  # noqa: BLE001
            print(json.dumps({"probe": fn.__name__, "error": repr(e)[:400]}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
