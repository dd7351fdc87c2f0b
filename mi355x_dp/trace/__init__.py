"""Tracing / profiling: the reference relies on SageMaker Debugger's
ProfilerReport (disabled inside the job) -- here:

* ``StepTimer``      -- per-phase GPU time with HIP events (data / forward / backward /
                        optimizer / comm-wait), negligible overhead, summarised per run;
* ``PhaseReport``    -- wall-clock phases of a job (initialization / training loop /
                        finalization) printed like the Debugger profiling report;
* ``python -m mi355x_dp.trace -- <cmd>`` -- runs ``rocprofv3 --kernel-trace --stats`` on a
  command and writes a markdown per-kernel summary (what profiles/*.md are made from).
"""
from __future__ import annotations

import contextlib
import json
import os
import time
from collections import defaultdict
from typing import Dict, List

import torch


class StepTimer:
    """``with timer.phase("forward"): ...`` -- GPU time per phase via events on the current stream."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._pending: List = []
        self.totals: Dict[str, float] = defaultdict(float)
        self.counts: Dict[str, int] = defaultdict(int)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            t0 = time.perf_counter()
            yield
            self.totals[name] += (time.perf_counter() - t0) * 1000
            self.counts[name] += 1
            return
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        yield
        e.record()
        self._pending.append((name, s, e))

    def flush(self):
        if self._pending:
            torch.cuda.synchronize()
            for name, s, e in self._pending:
                self.totals[name] += s.elapsed_time(e)
                self.counts[name] += 1
            self._pending = []

    def summary(self) -> Dict[str, Dict[str, float]]:
        self.flush()
        return {k: {"total_ms": round(v, 3), "calls": self.counts[k], "avg_ms": round(v / max(1, self.counts[k]), 3)}
                for k, v in self.totals.items()}


class PhaseReport:
    """Job-level phases, printed in the spirit of the Debugger ProfilerReport."""

    def __init__(self):
        self.t0 = time.time()
        self.marks: List = [("start", self.t0)]

    def mark(self, name: str):
        self.marks.append((name, time.time()))

    def report(self) -> Dict[str, float]:
        out = {}
        for (a, ta), (b, tb) in zip(self.marks, self.marks[1:]):
            out[b] = round(tb - ta, 3)
        out["total"] = round(self.marks[-1][1] - self.t0, 3)
        return out

    def print(self, file=None):
        r = self.report()
        print("Profiling report (phases, seconds): " + json.dumps(r), file=file, flush=True)
        return r


def rocprof_cmd(cmd: List[str], out_dir: str, name: str = "run") -> List[str]:
    """The rocprofv3 invocation used for kernel summaries (kernel trace + stats, csv)."""
    return ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", out_dir, "-o", name, "--", *cmd]
