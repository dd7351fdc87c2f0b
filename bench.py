#!/usr/bin/env python
"""Headline benchmark: ResNet-50 bf16 data-parallel training throughput (images/s,
whole job) on synthetic ImageNet-shaped data, 1..8 MI355X (BASELINE.json metric).

    python bench.py --gpus N --steps K --warmup W
    (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...)

Every timed step is a full training step through the framework's own engine:
GPU input pipeline (uint8 -> random flip + normalize -> bf16 NHWC), forward
(MFMA implicit-GEMM convs, fused BN/ReLU/residual, maxpool, GAP, fc), fused
cross-entropy, backward (dgrad/wgrad MFMA kernels, BN backward), bucketed
gradient all-reduce over RCCL overlapped with backward, fused flat SGD
(momentum 0.9, weight decay 1e-4).  Weak scaling: fixed per-GPU batch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--model", default="resnet50")
    p.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--num-classes", type=int, default=1000)
    p.add_argument("--lr", type=float, default=0.01)  # reference hyperparameter (nb2:110)
    p.add_argument("--backend", default=os.environ.get("MI355X_DP_BACKEND", "nccl"))
    p.add_argument("--bucket-mb", type=float, default=None)
    p.add_argument("--force-comm", action="store_true",
                   help="create the process group and issue every bucket collective even at N=1 "
                        "(comm-stream / overlap traces on one GPU); the headline N=1 run leaves it off")
    p.add_argument("--grad-comm", default=os.environ.get("MI355X_DP_GRAD_COMM", "fp32"), choices=("fp32", "bf16"),
                   help="gradient all-reduce dtype (bf16: half the bytes; fp32 master weights either way)")
    p.add_argument("--wgrad-stream", type=int, default=int(os.environ.get("MI355X_DP_WGRAD_STREAM", "1")),
                   choices=(0, 1), help="conv weight gradients on a side HIP stream (overlap with data gradients)")
    p.add_argument("--shard-optimizer", action="store_true",
                   default=os.environ.get("MI355X_DP_SHARD_OPTIMIZER", "0") == "1",
                   help="SMDDP balanced shards: reduce-scatter gradients, shard-local SGD, all-gather parameters")
    p.add_argument("--calibrate-comm", action="store_true",
                   help="size gradient buckets from an all-reduce alpha-beta fit measured at start-up")
    p.add_argument("--profile-steps", type=int, default=0, help="extra untimed steps after timing (rocprof)")
    p.add_argument("--graph", action="store_true",
                   help="replay the step as one captured HIP graph (launch-bound small-batch configs)")
    return p.parse_args()


def main():
    args = parse()
    if os.environ.get("MI355X_DP_BENCH_STACKS"):  # hang diagnosis: every rank dumps its Python stacks
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["MI355X_DP_BENCH_STACKS"]), repeat=True, file=sys.stderr)
    if args.graph and args.warmup < 2:
        args.warmup = 2  # the graph is captured during warmup, never inside the timed region
    import torch
    import torch.distributed as dist

    if int(os.environ.get("LOCAL_WORLD_SIZE", "1")) > max(1, torch.cuda.device_count()):
        # ranks share GPUs (multi-rank rehearsal on a small box): with the default 4 hardware queues
        # per process, 3+ processes oversubscribe the GPU's queue slots and the scheduler time-slices
        # them -- gloo's host-synchronised copies then crawl (profiles/multirank_rehearsal.md).
        # Must be set before the first HIP call (device_count() does not initialise HIP here).
        from mi355x_dp.utils import hwqueues
        if os.environ.get(hwqueues.AUTO_MARK) == "1":  # inherited from a one-rank-per-GPU parent
            os.environ.pop("GPU_MAX_HW_QUEUES", None)
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "1")
    else:
        # one rank per GPU: enough hardware queues that the compute, weight-gradient and comm
        # streams never share one (mi355x_dp/utils/hwqueues.py: 10.6k -> 12.6k img/s with a
        # process group on one MI355X)
        from mi355x_dp.utils import hwqueues
        hwqueues.ensure()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if rank == 0:
            print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    # one rank per GPU; more ranks than GPUs share them (gloo rehearsal of the multi-rank path on a
    # 1-GPU box -- RCCL itself refuses two ranks on one device)
    gpu = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    use_pg = world > 1 or args.force_comm
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
    kw["wgrad_stream"] = bool(args.wgrad_stream)
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
    x_static = torch.empty((B, 8, S, S), dtype=torch.bfloat16, device=dev, memory_format=torch.channels_last)

    def core():
        engine.zero_grad()
        out = engine(x_static)
        loss = cross_entropy(out, labels)
        loss.backward()
        opt.step()
        return loss

    graphed = None

    def step(i):
        nonlocal graphed
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
    if main_prio:
        torch.cuda.set_stream(torch.cuda.Stream(device=dev, priority=main_prio))
    t_w0 = time.time()
    for i in range(args.warmup):
        loss = step(i)
    torch.cuda.synchronize()
    first_loss = float(loss.detach()) if args.warmup else float("nan")
    t_w1 = time.time()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    torch.cuda.synchronize()
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

    comm_probe = None
    if world > 1 and os.environ.get("MI355X_DP_BENCH_COMM_PROBE", "1") == "1":
        # after the timed region: the fabric's measured collective times, recorded with the result
        # (feeds the bucket planner's alpha-beta model; all-reduce vs the balanced-shard RS + AG)
        from mi355x_dp.parallel.ddp import probe_collectives
        try:
            comm_probe = probe_collectives(device=dev)
        except Exception as e:  # never lose the measurement over the probe
            comm_probe = f"failed: {type(e).__name__}: {e}"

    for i in range(args.profile_steps):
        step(10_000 + i)
    torch.cuda.synchronize()

    total_images = world * B * args.steps
    value = total_images / elapsed
    if rank == 0:
        out = {
            "metric": "images/sec (whole node) ResNet-50 DDP" if args.model == "resnet50"
            else f"images/sec (whole node) {args.model} DDP",
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random uint8 ImageNet-shaped images, random labels; GPU flip+normalize pipeline; "
                    "random-init weights)",
            "config": {
                "model": args.model,
                "global_batch": B * world,
                "per_gpu_batch": B,
                "image_size": S,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "optimizer": "SGD(momentum=0.9, wd=1e-4), fp32 master weights, bf16 compute",
                "backend": args.backend if use_pg else "none",
                "comm_forced_at_world1": bool(args.force_comm and world == 1),
                "buckets": len(engine.buckets),
                "grad_comm": args.grad_comm,
                "shard_optimizer": bool(args.shard_optimizer),
                "wgrad_stream": bool(args.wgrad_stream),
                "hip_graph": bool(args.graph),
            },
            "loss_first_warmup": round(first_loss, 4),
            "loss_last": round(last_loss, 4),
            "warmup_s": round(t_w1 - t_w0, 2),
            "replicas_identical": replicas_ok,
            "comm_calibration": engine.calibration,
            "comm_probe": comm_probe,
            "bucket_launch_ms": [[b, round(nb / 2**20, 2), round(t / 1e3, 3)] for b, nb, t in engine.bucket_trace],
        }
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
