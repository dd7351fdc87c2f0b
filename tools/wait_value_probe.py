#!/usr/bin/env python
"""Does a command-processor gate (hipStreamWaitValue32 on signal memory, misc.hip mi_flag_wait) work
on this gfx950 / ROCm stack, and does it hold a CU while it waits?  (replace the
spinning mi_flag_gate kernel.)

A high-priority "gate" stream waits for flag >= 1, then runs a marker kernel; a normal-priority
"main" stream runs ~20 ms of matmuls, then the flag bump kernel (what a replayed backward graph
does per bucket).  The host never blocks on the gate: it polls the marker's event with a deadline
and, past it, releases the gate with a stream write of the flag (so the probe cannot hang the box).
Prints one JSON line: supported, ok (marker after the bump, no release needed), the marker's delay
after the main stream's end.  Run it under `rocprofv3 --kernel-trace` to see whether the runtime
launched a polling kernel for the wait.

    python tools/wait_value_probe.py
"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    lib = _lib.load(True)
    out = {"supported": int(lib.mi_wait_value_supported())}
    if not out["supported"]:
        print(json.dumps(out))
        return
    p = ctypes.c_void_p()
    _lib.check(lib.mi_signal_alloc(ctypes.byref(p)), "mi_signal_alloc")
    flag = p
    dev = torch.device("cuda", 0)
    gate = torch.cuda.Stream(device=dev, priority=-1)
    main_s = torch.cuda.Stream(device=dev, priority=0)
    rel = torch.cuda.Stream(device=dev, priority=-1)
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    marker = torch.zeros(1, device=dev)
    t0 = torch.cuda.Event(enable_timing=True)
    main_end, gate_open = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    t0.record(main_s)
    # the gate first: enqueued before the producer, as the engine enqueues gates before a replay
    with torch.cuda.stream(gate):
        _lib.check(lib.mi_flag_wait(flag, 1, ctypes.c_void_p(gate.cuda_stream)), "mi_flag_wait")
        gate_open.record(gate)
        marker.add_(1.0)
    with torch.cuda.stream(main_s):
        for _ in range(80):
            a = a @ a * 1e-3
        main_end.record(main_s)
        lib.mi_flag_bump(flag, ctypes.c_void_p(main_s.cuda_stream))
    deadline = time.time() + 10.0
    released = False
    while not gate_open.query():
        if time.time() > deadline:
            lib.mi_flag_release(flag, 1 << 30, ctypes.c_void_p(rel.cuda_stream))
            released = True
            break
        time.sleep(0.001)
    torch.cuda.synchronize()
    out.update({"released_by_host": released, "marker": float(marker.item()),
                "main_ms": round(t0.elapsed_time(main_end), 3), "gate_open_ms": round(t0.elapsed_time(gate_open), 3)})
    out["ok"] = (not released) and out["marker"] == 1.0 and out["gate_open_ms"] >= out["main_ms"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
