"""Graphed engine at world size W > 1: every rank runs the
reference's loop shape (ResNet-18, 1000-class head, batch 32 at 32x32, stock optim.SGD, through the
torch_smddp shim's engine-backed DistributedDataParallel) twice -- graphed (MI355X_DP_ENGINE_GRAPH=1:
forward + backward replayed as HIP graphs, bucket collectives behind per-bucket gates enqueued
before each replay -- IPC collectives cannot be captured) and eagerly --
and prints one JSON line: per-step losses of both runs, whether the final flat fp32 parameters are
bit-identical between the runs, the replica checksum of every rank, and the gate trace of the last
graphed step (ms from the replay's start at which each bucket's collective was released, and the ms
at which the replayed backward ended).  Launched by tests/test_gpu_integration.py through the
native launcher with IPC-only smddp (ranks may share one GPU), or -- on a box with >= 2 GPUs -- over
RCCL (GRAPHED_BACKEND=nccl, or smddp with MI355X_DP_SMDDP_IPC_ONLY=0), where the collectives are
captured into the backward graph (comm mode "capture")."""
import json
import os
import sys

os.environ.setdefault("MI355X_DP_WGRAD_STREAM", "0")  # single stream: eager == replay kernel for kernel
os.environ["MI355X_DP_GATE_TRACE"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.append(os.path.join(ROOT, "compat"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import smdistributed.dataparallel.torch.torch_smddp  # noqa: E402,F401  (installs the engine-backed DDP)

BACKEND = os.environ.get("GRAPHED_BACKEND", "smddp")  # "nccl": torch's ProcessGroupNCCL (RCCL)
if BACKEND == "nccl":
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
dist.init_process_group(backend=BACKEND)
r, w = dist.get_rank(), dist.get_world_size()
STEPS = int(os.environ.get("GRAPHED_STEPS", "8"))
# per-rank batch / image size (default: the reference's 32 at 32x32).  The gate-overlap check of the
# test runs a larger shape: at the reference shape the replayed backward (~0.9 ms) can finish before
# the host has even returned from launching the ~150-node graph, so no gate could open under it.
BATCH = int(os.environ.get("GRAPHED_BATCH", "32"))
SIZE = int(os.environ.get("GRAPHED_SIZE", "32"))


def run(mode):
    from mi355x_dp.models import get_model
    from mi355x_dp.parallel import step_graph
    step_graph.MODE = mode
    torch.manual_seed(0)
    model = get_model("resnet18", num_classes=1000).cuda()
    # GRAPHED_BCAST=0: no BN-buffer broadcast (its IPC kernel waits for the peer rank, which -- two
    # ranks time-slicing one GPU -- can lag by milliseconds and holds the comm stream in front of the
    # first gate; the gate-timing run measures the gates, not the peer's skew)
    ddp = torch.nn.parallel.DistributedDataParallel(
        model, broadcast_buffers=os.environ.get("GRAPHED_BCAST", "1") != "0")
    assert isinstance(ddp, torch.nn.parallel.DistributedDataParallel)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9)
    crit = torch.nn.CrossEntropyLoss().cuda()
    g = torch.Generator().manual_seed(11 + r)  # each rank its own shard of data
    losses = []
    for _ in range(STEPS):
        x = torch.randn(BATCH, 3, SIZE, SIZE, generator=g).cuda()
        y = torch.randint(0, 1000, (BATCH,), generator=g).cuda()
        opt.zero_grad()
        loss = crit(ddp(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    torch.cuda.synchronize()
    replays = sum(s.replays for s in getattr(ddp, "_graphs", {}).values())
    modes = sorted({s.comm_mode for s in getattr(ddp, "_graphs", {}).values()})
    return ddp, losses, replays, modes


eng_g, loss_g, replays, modes = run("1")
trace = eng_g.gate_trace_ms()
flat_g = eng_g.flat.data.clone()
eng_e, loss_e, replays_e, _ = run("0")
from mi355x_dp.parallel.health import ReplicaChecker  # noqa: E402
same = ReplicaChecker(eng_g)(force=True)
print(json.dumps({"rank": r, "world": w, "losses_graphed": loss_g, "losses_eager": loss_e, "replays": replays,
                  "replays_eager": replays_e, "gated": modes == ["gates"], "comm_modes": modes, "graphed_equals_eager": bool(torch.equal(flat_g,
                                                                                           eng_e.flat.data)),
                  "replicas_identical": bool(same), "buckets": len(eng_g.buckets),
                  "gate_open_ms": trace[0] if trace else None, "replay_end_ms": trace[1] if trace else None,
                  "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}),
      flush=True)
dist.destroy_process_group()
