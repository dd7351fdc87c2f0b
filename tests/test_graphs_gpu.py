"""HIP-graph replay of a whole training step (mi355x_dp.graphs) reproduces an eager step taken
from the same state (weights, momentum, BN statistics) on the same input."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_graphed_step_matches_eager():
    from mi355x_dp.graphs import GraphedStep
    from mi355x_dp.models import get_model
    from mi355x_dp.ops import augment, cross_entropy
    from mi355x_dp.parallel import DataParallel, FlatSGD
    torch.manual_seed(0)
    eng = DataParallel(get_model("resnet18", num_classes=10).cuda())
    opt = FlatSGD(eng, lr=0.01, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device="cuda").manual_seed(3)
    imgs = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, device="cuda", generator=g)
    labels = torch.randint(0, 10, (32,), device="cuda", generator=g)
    mean, std = (0.49, 0.48, 0.45), (0.2, 0.2, 0.2)
    x = torch.empty((32, 8, 32, 32), dtype=torch.bfloat16, device="cuda", memory_format=torch.channels_last)

    def core():
        eng.zero_grad()
        loss = cross_entropy(eng(x), labels)
        loss.backward()
        opt.step()
        return loss

    augment(imgs, 8, mean, std, pad=4, flip=True, seed=0, out=x)
    core()                                   # eager first step (optimizer first-step semantics)
    gs = GraphedStep(core, warmup=1)         # one more eager step on a side stream, then capture
    state = [eng.flat.data, eng.flat.bf16, opt.momentum_buf, eng.buffers.data]
    if eng.flat.bf16_t is not None:  # transposed dgrad copies of the conv weights
        state.append(eng.flat.bf16_t)
    snap = [t.clone() for t in state]

    augment(imgs, 8, mean, std, pad=4, flip=True, seed=7, out=x)
    loss_eager = float(core())
    p_eager = eng.flat.data.clone()
    for t, s in zip(state, snap):
        t.copy_(s)
    loss_graph = float(gs())
    torch.cuda.synchronize()
    assert gs.replays == 1
    assert loss_graph == pytest.approx(loss_eager, rel=1e-3)
    step_eager = (p_eager - snap[0]).abs().max()
    assert float((eng.flat.data - p_eager).abs().max()) <= 1e-2 * float(step_eager)


def test_bench_graph_fresh_process():
    """bench.py --graph in a fresh process: the eager steps before capture run with the weight-
    gradient side stream, the graph warm-up / capture single-stream on one stream -- every lazily
    sized native workspace must exist before the capture (regression: a capture-time allocation
    invalidated the capture when only the side stream's workspace had been sized)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--model", "resnet18", "--batch", "32",
                        "--image-size", "32", "--num-classes", "10", "--steps", "5", "--warmup", "2", "--graph"],
                       capture_output=True, text=True, timeout=300, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["config"]["hip_graph"] is True and out["value"] > 0
