#!/usr/bin/env python
"""Headline benchmark: ResNet-50 bf16 data-parallel training throughput (images/s,
whole job) on synthetic ImageNet-shaped data, 1..8 MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W
        N>1 without a launcher: bench.py spawns the N ranks itself through the native
        launcher (csrc/launch/launcher.cpp, the mpirun/smddprun replacement, reference
        nb2:284 `mpirun -np 8 ... smddprun`) and relays rank 0's JSON line and the job's
        exit code.  The parent makes no HIP call.
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
        (or any launcher that sets WORLD_SIZE / RANK / LOCAL_RANK): one rank per process.

Every rank checks that the process group it joined really has --gpus ranks (exit 3 otherwise,
never a world-1 number under an N-GPU label) and the JSON line reports ``ranks_seen`` and the
collective backend (RCCL version for ``nccl``).

Every timed step is a full training step through the framework's own engine:
GPU input pipeline (uint8 -> random flip + normalize -> bf16 NHWC), forward
(MFMA implicit-GEMM convs, fused BN/ReLU/residual, maxpool, GAP, fc), fused
cross-entropy, backward (dgrad/wgrad MFMA kernels, BN backward), bucketed
gradient all-reduce over RCCL overlapped with backward, fused flat SGD
(momentum 0.9, weight decay 1e-4).  Weak scaling: fixed per-GPU batch.

``--device cpu`` runs the same distributed code path (bucket planner, C++ reducer, gloo
collectives, comm probe, replica check) on CPU ranks -- a rehearsal of the world-8 path for
tests on machines without a GPU; its numbers are not GPU measurements.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
EXIT_WORLD_MISMATCH = 3


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--model", default="resnet50")
    p.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--num-classes", type=int, default=1000)
    p.add_argument("--lr", type=float, default=0.01)  # reference hyperparameter (nb2:110)
    p.add_argument("--backend", default=os.environ.get("MI355X_DP_BACKEND"),
                   help="collective backend (default: nccl = RCCL on cuda, gloo on cpu)")
    p.add_argument("--device", default="cuda", choices=("cuda", "cpu"),
                   help="cpu: rehearse the distributed path on CPU ranks (tests; not a GPU number)")
    p.add_argument("--bucket-mb", type=float, default=None)
    p.add_argument("--comm-emulate", type=int, default=int(os.environ.get("MI355X_DP_COMM_EMULATE", "0") or 0),
                   help="world 1: run every gradient all-reduce as one rank of an N-rank ring on the smddp "
                        "backend's comm stream (memory traffic, CU footprint, xGMI-paced duration; "
                        "mi_ring_emulate) -- implies --backend smddp --force-comm")
    p.add_argument("--force-comm", action="store_true",
                   help="create the process group and issue every bucket collective even at N=1 "
                        "(comm-stream / overlap traces on one GPU); the headline N=1 run leaves it off")
    p.add_argument("--grad-comm", default=os.environ.get("MI355X_DP_GRAD_COMM", "fp32"), choices=("fp32", "bf16"),
                   help="gradient all-reduce dtype (bf16: half the bytes; fp32 master weights either way)")
    p.add_argument("--wgrad-stream", default=os.environ.get("MI355X_DP_WGRAD_STREAM", "auto"),
                   choices=("auto", "0", "1"),
                   help="weight gradients on a side HIP stream (overlap with data gradients); auto: on for "
                        "BatchNorm conv nets, off for GEMM-bound models (mi355x_dp.parallel.ddp.WGRAD_STREAM)")
    p.add_argument("--shard-optimizer", action="store_true",
                   default=os.environ.get("MI355X_DP_SHARD_OPTIMIZER", "0") == "1",
                   help="SMDDP balanced shards: reduce-scatter gradients, shard-local SGD, all-gather parameters")
    p.add_argument("--calibrate-comm", action="store_true",
                   help="size gradient buckets from an all-reduce alpha-beta fit measured at start-up")
    p.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps after timing (rocprof)")
    p.add_argument("--graph", action="store_true",
                   help="replay the step as one captured HIP graph (launch-bound small-batch configs)")
    p.add_argument("--launcher", default=os.environ.get("MI355X_DP_BENCH_LAUNCHER", "native"),
                   choices=("native", "torchrun"), help="how --gpus N > 1 spawns its ranks without WORLD_SIZE")
    a = p.parse_args(argv)
    if a.comm_emulate > 1:
        a.backend, a.force_comm = "smddp", True
        os.environ["MI355X_DP_COMM_EMULATE"] = str(a.comm_emulate)
    if a.backend is None:
        a.backend = "nccl" if a.device == "cuda" else "gloo"
    return a


# ------------------------------------------------------------------ self-spawn (parent process)
def spawn_ranks(args, argv) -> int:
    """Run this script as ``args.gpus`` ranks on this node and relay the result.

    The parent never initialises HIP (``torch.cuda.device_count`` does not on this stack; no other
    torch.cuda call is made).  Child stdout lines that parse as the result JSON are printed on this
    process's stdout (exactly one, from rank 0); every other line goes to stderr.  Returns the job
    exit code: the first failing rank's (the native launcher aborts the others), 0 otherwise."""
    n = args.gpus
    if args.device == "cuda":
        try:
            import torch
            ngpu = torch.cuda.device_count()
        except Exception:
            ngpu = 0
        if ngpu == 0:
            print("[bench] --gpus N > 1 needs GPUs (or --device cpu for a CPU rehearsal)", file=sys.stderr)
            return 2
        if n > ngpu and args.backend == "nccl":
            print(f"[bench] --gpus {n} > {ngpu} visible GPUs: RCCL needs one device per rank "
                  f"(use --backend gloo to rehearse {n} ranks sharing the GPUs)", file=sys.stderr)
            return 2
    from mi355x_dp.launch import NATIVE_LAUNCHER, compat_pythonpath, free_port
    port = int(os.environ.get("MASTER_PORT") or free_port())
    script = [sys.executable, os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env["PYTHONUNBUFFERED"] = "1"  # rank output relayed line by line
    env["PYTHONPATH"] = compat_pythonpath(env.get("PYTHONPATH"))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["MI355X_DP_BENCH_SPAWNED"] = args.launcher
    if args.launcher == "native" and os.path.exists(NATIVE_LAUNCHER):
        cmd = [NATIVE_LAUNCHER, "--nproc", str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
               "--"] + script
    else:
        env["MI355X_DP_BENCH_SPAWNED"] = "torchrun"
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr=127.0.0.1", f"--master-port={port}"] + script[1:]
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    results = 0
    for line in proc.stdout:
        if _is_result(line):
            results += 1
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    rc = proc.wait()
    if rc == 0 and results != 1:
        print(f"[bench] ranks exited 0 but {results} result lines were printed", file=sys.stderr)
        return 1
    return rc


def _is_result(line: str) -> bool:
    s = line.strip()
    if not (s.startswith("{") and '"metric"' in s):
        return False
    try:
        return "value" in json.loads(s)
    except ValueError:
        return False


def _backend_info(dist, backend: str):
    """(backend name as the process group reports it, collective library version)"""
    name = str(dist.get_backend())
    lib = None
    if name == "nccl":
        try:
            import torch
            v = torch.cuda.nccl.version()
            lib = "RCCL " + (".".join(str(x) for x in v) if isinstance(v, tuple) else str(v))
        except Exception:
            lib = "RCCL"
    elif name == "gloo":
        lib = "gloo"
    else:
        lib = name
    return name, lib


# --------------------------------------------------------------------------------- rank process
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args, argv))
    if os.environ.get("MI355X_DP_BENCH_STACKS"):  # hang diagnosis: every rank dumps its Python stacks
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["MI355X_DP_BENCH_STACKS"]), repeat=True, file=sys.stderr)
    if args.graph and args.warmup < 2:
        args.warmup = 2  # the graph is captured during warmup, never inside the timed region

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # never report a number for a world the caller did not ask for
        print(f"[bench] rank {rank}: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks; "
              "refusing to run", file=sys.stderr)
        sys.exit(EXIT_WORLD_MISMATCH)
    cuda = args.device == "cuda"

    import torch
    import torch.distributed as dist

    if cuda:
        # hardware queues per process, sized before the first HIP call (utils/hwqueues.py): one
        # rank per GPU gets enough queues that the compute, weight-gradient and comm streams never
        # share one; ranks sharing a GPU (multi-rank rehearsal) get one each
        from mi355x_dp.utils import hwqueues
        hwqueues.ensure()
        # one rank per GPU; more ranks than GPUs share them (gloo rehearsal of the multi-rank path on
        # a 1-GPU box -- RCCL itself refuses two ranks on one device)
        gpu = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(gpu)
        dev = torch.device("cuda", gpu)
    else:
        dev = torch.device("cpu")
        torch.set_num_threads(max(1, int(os.environ.get("MI355X_DP_BENCH_CPU_THREADS", "1"))))

    def sync():
        if cuda:
            torch.cuda.synchronize()

    use_pg = world > 1 or args.force_comm
    ranks_seen, backend_name, comm_lib = 1, "none", None
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if args.backend == "smddp":
            sys.path.append(os.path.join(ROOT, "compat"))
            import smdistributed.dataparallel.torch.torch_smddp  # noqa: F401  (registers 'smddp')
        pg_options = None
        if args.backend == "nccl" and os.environ.get("MI355X_DP_NCCL_HIPRIO", "1") == "1":
            # RCCL kernels on a high-priority stream (as the native smddp backend does): with the
            # compute and weight-gradient streams filling the CUs, the bucket all-reduces are
            # dispatched first instead of queueing behind backward kernels
            pg_options = dist.ProcessGroupNCCL.Options()
            pg_options.is_high_priority_stream = True
        dist.init_process_group(backend=args.backend, device_id=dev if args.backend == "nccl" else None,
                                pg_options=pg_options)
        ranks_seen = dist.get_world_size()
        backend_name, comm_lib = _backend_info(dist, args.backend)
        if ranks_seen != args.gpus and not (args.force_comm and args.gpus == 1 and ranks_seen == 1):
            print(f"[bench] rank {rank}: process group has {ranks_seen} ranks, --gpus {args.gpus}", file=sys.stderr)
            sys.exit(EXIT_WORLD_MISMATCH)

    from mi355x_dp.models import get_model
    from mi355x_dp.ops import augment, cross_entropy
    from mi355x_dp.parallel import DataParallel, FlatSGD

    torch.manual_seed(1234 + rank)
    model = get_model(args.model, num_classes=args.num_classes).to(dev)
    kw = {}
    if args.bucket_mb:
        kw["bucket_cap_mb"] = args.bucket_mb
    if args.force_comm:
        kw["force_comm"] = True
    kw["grad_comm"] = args.grad_comm
    kw["wgrad_stream"] = "auto" if args.wgrad_stream == "auto" else args.wgrad_stream == "1"
    if args.calibrate_comm:
        kw["calibrate"] = True
    kw["shard_optimizer"] = bool(args.shard_optimizer)
    engine = DataParallel(model, **kw)
    opt = FlatSGD(engine, lr=args.lr, momentum=0.9, weight_decay=1e-4)

    B, S = args.batch, args.image_size
    g = torch.Generator(device=dev)
    g.manual_seed(rank)
    images = torch.randint(0, 256, (B, S, S, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, args.num_classes, (B,), dtype=torch.int64, device=dev, generator=g)

    pad = 4 if S <= 64 else 0  # CIFAR-style random crop for small images (reference transforms)
    x_static = (torch.empty((B, 8, S, S), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)
                if cuda else None)

    def core():
        engine.zero_grad()
        out = engine(x_static)
        loss = cross_entropy(out, labels)
        loss.backward()
        opt.step()
        return loss

    graphed = None

    def step(i):
        nonlocal graphed, x_static
        if not cuda:  # CPU rehearsal: the op library's ATen fallback returns a fresh fp32 NCHW batch
            x_static = augment(images, 3, IMAGENET_MEAN, IMAGENET_STD, pad=pad, flip=True, seed=i)
            return core()
        augment(images, 8, IMAGENET_MEAN, IMAGENET_STD, pad=pad, flip=True, seed=i, out=x_static)  # 3 ch + 5 zero
        if args.graph and i >= 1:  # capture after one eager step (optimizer first-step semantics)
            if graphed is None:
                from mi355x_dp.graphs import GraphedStep
                graphed = GraphedStep(core, warmup=1)
            return graphed()
        return core()

    # MI355X_DP_MAIN_PRIORITY=-1: the training step's compute stream at high priority (its
    # workgroups dispatched ahead of the weight-gradient side stream's)
    main_prio = int(os.environ.get("MI355X_DP_MAIN_PRIORITY", "0"))
    if main_prio and cuda:
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=main_prio))
    t_w0 = time.time()
    for i in range(args.warmup):
        loss = step(i)
    sync()
    first_loss = float(loss.detach()) if args.warmup else float("nan")
    t_w1 = time.time()

    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    sync()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    last_loss = float(loss.detach())
    replicas_ok = None
    if world > 1:  # after the timed region: every rank's flat fp32 master weights bit-identical?
        from mi355x_dp.parallel.health import ReplicaChecker, ReplicaDivergence
        try:
            replicas_ok = ReplicaChecker(engine)(force=True)
        except ReplicaDivergence as e:
            print(f"[bench] {e}", file=sys.stderr)
            replicas_ok = False

    comm_timeline = None
    if engine.reducer is not None and engine.comm_on and cuda and not args.graph:
        # after the timed region, one more step with GPU events around every bucket collective
        # (every rank runs it, so the collectives still match): when each bucket became ready on the
        # producing stream, when its collective ended on the comm stream, when the backward's
        # kernels ended -- the overlap record in device time, not host launch time
        # (two untimed steps first, so the host runs ahead of the GPU as in the timed loop: right
        # after a synchronize the device would idle on the host's first launches of the step)
        step(20_000)
        step(20_001)
        engine.reducer.gpu_timing = True
        step(20_002)
        sync()
        comm_timeline = _timeline(engine)
        engine.reducer.gpu_timing = False

    comm_probe = None
    if world > 1 and os.environ.get("MI355X_DP_BENCH_COMM_PROBE", "1") == "1":
        # after the timed region: the fabric's measured collective times, recorded with the result
        # (feeds the bucket planner's alpha-beta model; all-reduce vs the balanced-shard RS + AG)
        from mi355x_dp.parallel.ddp import probe_collectives
        sizes = tuple(float(s) for s in os.environ.get("MI355X_DP_BENCH_PROBE_MB", "0.25,4,32,128").split(","))
        try:
            comm_probe = probe_collectives(device=dev, sizes_mb=sizes)
        except Exception as e:  # never lose the measurement over the probe
            comm_probe = f"failed: {type(e).__name__}: {e}"

    for i in range(args.profile_steps):
        step(10_000 + i)
    sync()

    total_images = world * B * args.steps
    value = total_images / elapsed
    if use_pg:
        dist.destroy_process_group()
        use_pg = False
    smddp_job = None
    if rank == 0 and world > 1 and args.backend != "smddp" and os.environ.get(
            "MI355X_DP_BENCH_SMDDP_JOB", "1" if cuda else "0") == "1":
        # after the timed region, as its own N-rank job: the same training step through the native
        # `smddp` c10d backend (csrc/comm/smddp_backend.cpp, the reference's backend name,
        # gpu.py:17-23 / nb2:781,1223) -- so every multi-GPU run also exercises the product path,
        # while the headline keeps the path most likely to succeed
        if cuda and world > torch.cuda.device_count():
            # ranks sharing a device (one-GPU rehearsals): RCCL refuses two ranks on one GPU
            smddp_job = "skipped: ranks share a device"
        else:
            if cuda:
                torch.cuda.empty_cache()
            smddp_job = run_child_bench(world, args, "smddp")
    secondary = None
    if (rank == 0 and world == 1 and cuda and args.model == "resnet50" and not args.force_comm
            and os.environ.get("MI355X_DP_BENCH_SECONDARY", "1") == "1"):
        # after the timed region, each as its own process: the other BASELINE.json configs' models
        # (ResNet-152, ViT-B/16, same per-GPU batch) on this same box, so every driver run records
        # them too -- a failure or timeout there cannot cost the headline measurement
        torch.cuda.empty_cache()
        secondary = {m: run_child_bench(1, args, args.backend, model=m, timeout_s=180)
                     for m in ("resnet152", "vit_b_16")}
    emulated = None
    if (rank == 0 and world == 1 and cuda and not args.force_comm
            and os.environ.get("MI355X_DP_BENCH_EMULATE", "1") == "1"):
        # after the timed region, as its own process: the same step with every bucket all-reduce run
        # as one rank of an 8-rank ring on the smddp comm stream (mi_ring_emulate: the rank's memory
        # traffic on 32 resident workgroups, paced to xGMI time) -- at world 1 RCCL launches nothing,
        # so this is the single-GPU estimate of what an 8-GPU gradient exchange costs the backward
        # (VERDICT r5 item 3); the headline above stays the plain world-1 step
        torch.cuda.empty_cache()
        emulated = run_child_bench(1, args, "smddp", timeout_s=180, extra=["--comm-emulate", "8"])
    ipc_probe = None
    if (rank == 0 and world > 1 and cuda and world <= torch.cuda.device_count()
            and os.environ.get("MI355X_DP_BENCH_IPC_PROBE", "1") == "1"):
        # after the timed region, as its own job: the native smddp backend's IPC one-/two-shot
        # all-reduce against RCCL per size on this fabric, and the per-size path choice it implies
        ipc_probe = run_ipc_probe(world)
    if rank == 0:
        out = {
            "metric": "images/sec (whole node) ResNet-50 DDP" if args.model == "resnet50"
            else f"images/sec (whole node) {args.model} DDP",
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if cuda else "fp32",
            "data": "synthetic (random uint8 ImageNet-shaped images, random labels; GPU flip+normalize pipeline; "
                    "random-init weights)" + ("" if cuda else "; CPU REHEARSAL, not a GPU measurement"),
            "config": {
                "model": args.model,
                "global_batch": B * world,
                "per_gpu_batch": B,
                "image_size": S,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "optimizer": "SGD(momentum=0.9, wd=1e-4), fp32 master weights, " + ("bf16 compute" if cuda else "fp32 compute"),
                "backend": backend_name,
                "comm_library": comm_lib,
                "launcher": os.environ.get("MI355X_DP_BENCH_SPAWNED", "external" if world > 1 else "none"),
                "device": args.device,
                "comm_forced_at_world1": bool(args.force_comm and world == 1),
                "buckets": len(engine.buckets),
                "grad_comm": args.grad_comm,
                "shard_optimizer": bool(args.shard_optimizer),
                "wgrad_stream": engine.wgrad_stream is not None,
                "hip_graph": bool(args.graph),
                "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
            },
            "loss_first_warmup": round(first_loss, 4),
            "loss_last": round(last_loss, 4),
            "warmup_s": round(t_w1 - t_w0, 2),
            "replicas_identical": replicas_ok,
            "comm_calibration": engine.calibration,
            "comm_probe": comm_probe,
            "ipc_probe": ipc_probe,
            "smddp_job": smddp_job,
            "secondary_models": secondary,
            "emulated_comm_dp8": emulated,
            "comm_emulated_world": args.comm_emulate if args.comm_emulate > 1 else None,
            # GPU event times (ms from the forward's start) of one step after the timed region
            "comm_timeline": comm_timeline,
            "bucket_launch_ms": comm_timeline["buckets"] if comm_timeline else None,
            "comm_exposed_ms": comm_timeline["comm_exposed_ms"] if comm_timeline else None,
            # host clock when each bucket's collective was handed to the backend (not overlap evidence)
            "bucket_issue_host_ms": [[b, round(nb / 2**20, 2), round(t / 1e3, 3)] for b, nb, t in engine.bucket_trace],
        }
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.destroy_process_group()


def _timeline(engine):
    """The reducer's GPU timeline of the last step (csrc/ddp/reducer.cpp ``gpu_trace``): per bucket
    [bucket, MB, ready_ms, start_ms, end_ms] -- start = max(ready, previous collective's end), as
    collectives run one after another on the comm stream -- plus the end of the backward's kernels and
    ``comm_exposed_ms`` = last collective end - backward end (>= 0): the communication the step waited
    for after its compute."""
    bwd_end, rows = engine.reducer.gpu_trace()
    if not rows or bwd_end < 0:
        return None
    out, prev_end = [], 0.0
    for b, nbytes, ready, end in rows:
        start = max(ready, prev_end)
        out.append([b, round(nbytes / 2**20, 2), round(ready, 3), round(start, 3), round(end, 3)])
        prev_end = end
    last_end = max(r[4] for r in out)
    return {"ref": "forward start of the step", "bwd_end_ms": round(bwd_end, 3), "buckets": out,
            "comm_ms": round(sum(r[4] - r[3] for r in out), 3),
            "comm_exposed_ms": round(max(0.0, last_end - bwd_end), 3)}


def _child_env():
    from mi355x_dp.launch import compat_pythonpath
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_PORT",
                        "MASTER_ADDR", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
                        "TORCHELASTIC_MAX_RESTARTS", "MI355X_DP_BENCH_SPAWNED")}
    env["PYTHONPATH"] = compat_pythonpath(env.get("PYTHONPATH"))
    env["PYTHONUNBUFFERED"] = "1"
    return env


def run_child_bench(world: int, args, backend: str, timeout_s: int = 150, model: str = None, extra=()):
    """``bench.py`` again as a fresh N-rank job (native launcher) through ``backend``, a few steps of
    the same configuration (or of ``model``), started by rank 0 after the benchmark finished (a
    failure cannot cost the measurement).  Returns its img/s, ranks seen, backend, replica check and
    step time."""
    from mi355x_dp.launch import NATIVE_LAUNCHER, free_port
    if not os.path.exists(NATIVE_LAUNCHER):
        return "skipped: native launcher not built"
    env = _child_env()
    env["MI355X_DP_BENCH_SMDDP_JOB"] = "0"   # no nested child jobs
    env["MI355X_DP_BENCH_IPC_PROBE"] = "0"
    env["MI355X_DP_BENCH_COMM_PROBE"] = "0"
    env["MI355X_DP_BENCH_SECONDARY"] = "0"
    env["MI355X_DP_BENCH_SPAWNED"] = "native"
    steps = max(1, min(args.steps, int(os.environ.get("MI355X_DP_BENCH_SMDDP_STEPS", "10"))))
    # a secondary model keeps its own wgrad-stream policy (auto: off for the GEMM-bound ViT)
    wgs = "auto" if model else str(args.wgrad_stream)
    cmd = [NATIVE_LAUNCHER, "--nproc", str(world), "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           "--", sys.executable, os.path.abspath(__file__), "--gpus", str(world), "--steps", str(steps),
           "--warmup", str(min(max(args.warmup, 1), 3)), "--model", model or args.model, "--batch", str(args.batch),
           "--image-size", str(args.image_size), "--num-classes", str(args.num_classes), "--backend", backend,
           "--device", args.device, "--grad-comm", args.grad_comm, "--wgrad-stream", wgs]
    if args.shard_optimizer:
        cmd.append("--shard-optimizer")
    cmd += list(extra)
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        out, err = proc.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        proc.terminate()  # the launcher forwards it to every rank (abort-all), then SIGKILLs them
        try:
            proc.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.communicate()
        return f"failed: timeout after {timeout_s} s"
    for line in out.splitlines():
        if _is_result(line):
            d = json.loads(line)
            return {"model": d["config"]["model"], "backend": d["config"]["backend"],
                    "comm_library": d["config"]["comm_library"], "img_s": d["value"],
                    "ms_per_step": d["ms_per_step"], "steps": d["steps"], "warmup": d["warmup"],
                    "per_gpu_batch": d["config"]["per_gpu_batch"], "ranks_seen": d["ranks_seen"],
                    "replicas_identical": d["replicas_identical"], "buckets": d["config"]["buckets"],
                    "comm_emulated_world": d.get("comm_emulated_world"),
                    "comm_exposed_ms": d.get("comm_exposed_ms"), "comm_timeline": d.get("comm_timeline")}
    return f"failed: rc={proc.returncode}: {(err or out)[-400:]}"


def run_ipc_probe(world: int, timeout_s: int = 120):
    """The smddp IPC-vs-RCCL path table of this node (tools/ipc_probe.py), as a separate N-rank job
    started by rank 0 after the benchmark finished: a probe failure cannot cost the measurement."""
    from mi355x_dp.launch import NATIVE_LAUNCHER, compat_pythonpath, free_port
    if not os.path.exists(NATIVE_LAUNCHER):
        return "skipped: native launcher not built"
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_PORT",
                        "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS")}
    env["PYTHONPATH"] = compat_pythonpath(env.get("PYTHONPATH"))
    cmd = [NATIVE_LAUNCHER, "--nproc", str(world), "--master-addr", "127.0.0.1", "--master-port",
           str(free_port()), "--", sys.executable, os.path.join(ROOT, "tools", "ipc_probe.py")]
    # the launcher forwards SIGTERM to every rank (abort-all) and SIGKILLs them after its grace
    # period: a hung probe never leaves orphaned GPU processes behind
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        out, err = proc.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        proc.terminate()
        try:
            proc.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.communicate()
        return f"failed: timeout after {timeout_s} s"
    for line in out.splitlines():
        if line.startswith('{"ipc_probe"'):
            return json.loads(line)["ipc_probe"]
    return f"failed: rc={proc.returncode}: {(err or out)[-300:]}"


if __name__ == "__main__":
    main()
