"""bench.py's multi-rank contract on CPU ranks (no GPU): self-spawn of --gpus N ranks through the
native launcher (or torchrun), relay of rank 0's single JSON line and the job exit code, refusal
of a world size that differs from --gpus, and the world-8 distributed path (bucket planner, C++
reducer, gloo collectives, comm probe, replica check) as 8 gloo ranks -- the shape of the
reference's 8-rank job (nb2:284 `mpirun -np 8`, 8-rank communicators nb2:781, nb2:1223)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--device", "cpu", "--model", "resnet18", "--image-size", "32", "--batch", "2", "--steps", "1",
         "--warmup", "1"]


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    env["MI355X_DP_BENCH_PROBE_MB"] = "0.25,4"
    env.update(kw)
    return env


def _run(args, env=None, timeout=600):
    p = subprocess.run([sys.executable, BENCH] + args, env=env or _env(), cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    return p.returncode, lines, p.stderr


def _check(lines, n):
    assert len(lines) == 1, lines  # exactly one JSON line on stdout, nothing else
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranks_seen"] == n
    assert d["config"]["parallelism"] == f"dp{n}" and d["config"]["global_batch"] == 2 * n
    assert d["config"]["backend"] == "gloo"
    assert d["replicas_identical"] is True
    assert isinstance(d["comm_probe"], list) and [r["mb"] for r in d["comm_probe"]] == [0.25, 4.0]
    assert d["value"] > 0 and d["steps"] == 1
    return d


def test_self_spawn_native_launcher_world2():
    rc, lines, err = _run(["--gpus", "2"] + SMALL)
    assert rc == 0, err[-3000:]
    d = _check(lines, 2)
    assert d["config"]["launcher"] == "native"


def test_self_spawn_torchrun_world2():
    rc, lines, err = _run(["--gpus", "2", "--launcher", "torchrun"] + SMALL)
    assert rc == 0, err[-3000:]
    assert _check(lines, 2)["config"]["launcher"] == "torchrun"


def test_world8_rehearsal_on_cpu_ranks():
    """The N=8 code path end to end: 8 ranks, planner + reducer + 8-rank gloo all-reduces, the
    post-timing comm probe (MAX over 8 ranks) and the bit-identical replica check."""
    rc, lines, err = _run(["--gpus", "8"] + SMALL)
    assert rc == 0, err[-3000:]
    d = _check(lines, 8)
    assert d["config"]["buckets"] >= 2
    # bucket launch trace: every bucket went to the comm stream in order during backward
    ids = [b for b, _, _ in d["bucket_issue_host_ms"] if b >= 0]
    assert d["comm_timeline"] is None  # GPU event timeline: CUDA engines only
    assert ids == list(range(d["config"]["buckets"]))


def test_world_size_mismatch_is_an_error():
    """An external launcher that started a different number of ranks than --gpus: every rank exits
    3 before doing any work, and no result line is printed."""
    rc, lines, err = _run(["--gpus", "2"] + SMALL, env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert rc == 3 and lines == [] and "refusing" in err


def test_failing_rank_propagates_exit_code():
    """A rank that dies (unknown model) fails the whole job with its exit code; no JSON is relayed."""
    rc, lines, err = _run(["--gpus", "2", "--device", "cpu", "--model", "no_such_model", "--steps", "1",
                           "--warmup", "0"])
    assert rc != 0 and lines == []


def test_spawn_refuses_rccl_with_more_ranks_than_gpus(monkeypatch):
    """The parent checks device count (no HIP init) and refuses an RCCL job with more ranks than GPUs."""
    sys.path.insert(0, ROOT)
    import importlib
    bench = importlib.import_module("bench")
    import torch
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    args = bench.parse(["--gpus", "2"])
    assert args.backend == "nccl"
    assert bench.spawn_ranks(args, ["--gpus", "2"]) == 2
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 0)
    assert bench.spawn_ranks(args, ["--gpus", "2"]) == 2


@pytest.mark.parametrize("line,ok", [
    ('{"metric": "m", "value": 1.0}', True),
    ('{"metric": "m"}', False),
    ('{"metric": "m", "value": ', False),
    ("[bench] note", False),
])
def test_result_line_detection(line, ok):
    sys.path.insert(0, ROOT)
    import importlib
    assert importlib.import_module("bench")._is_result(line) is ok


def test_post_timing_smddp_job_on_cpu_ranks():
    """after the timed region rank 0 starts the same step as a fresh N-rank job
    through the native `smddp` backend name (on CPU ranks it falls back to gloo) and reports it in
    the JSON line; the headline fields are the parent job's (backend gloo / nccl)."""
    rc, lines, err = _run(["--gpus", "2"] + SMALL, env=_env(MI355X_DP_BENCH_SMDDP_JOB="1"))
    assert rc == 0, err[-3000:]
    d = _check(lines, 2)
    j = d["smddp_job"]
    assert isinstance(j, dict), j
    assert j["backend"] == "smddp" and j["ranks_seen"] == 2 and j["replicas_identical"] is True, j
    assert j["img_s"] > 0 and j["buckets"] == d["config"]["buckets"]
