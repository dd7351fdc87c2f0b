"""Foreign-optimizer engine with graphed forward/backward (parallel/step_graph.py) == the same
engine run eagerly, for the reference script's loop shape (stock optim.SGD, CrossEntropyLoss,
fp32 NCHW batches of 32 at 32x32, a smaller last batch, eval passes in between)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(graph_mode, steps, monkeypatch, wgrad_stream=False):
    from mi355x_dp.models import get_model
    from mi355x_dp.parallel import DataParallel, step_graph
    monkeypatch.setattr(step_graph, "MODE", graph_mode)
    torch.manual_seed(0)
    model = get_model("resnet18", num_classes=1000).cuda()
    # wgrad_stream=False: every eager step on one stream like the (single-stream) replays, so the
    # same kernels with the same grids run in both runs and the results are bit-identical
    eng = DataParallel(model, foreign_optimizer=True, wgrad_stream=wgrad_stream)
    opt = torch.optim.SGD(eng.parameters(), lr=0.01, momentum=0.9)
    crit = torch.nn.CrossEntropyLoss().cuda()
    g = torch.Generator().manual_seed(5)
    losses = []
    for i in range(steps):
        n = 32 if i != steps - 2 else 10  # a short batch (an epoch's last) between full ones
        data = torch.randn(n, 3, 32, 32, generator=g).cuda()
        target = torch.randint(0, 10, (n,), generator=g).cuda()
        opt.zero_grad()
        out = eng(data)
        loss = crit(out, target)
        loss.backward()
        opt.step()
        losses.append(float(loss))
        if i == 4:  # an evaluation pass in the middle (eval mode, no grad): eager
            eng.eval()
            with torch.no_grad():
                eng(torch.randn(100, 3, 32, 32, generator=g).cuda())
            eng.train()
    torch.cuda.synchronize()
    graphs = getattr(eng, "_graphs", {})
    replays = sum(s.replays for s in graphs.values())
    return losses, eng.flat.data.clone(), eng.buffers.data.clone(), \
        [b.clone() for b in eng.buffers.others], replays


def test_graphed_engine_matches_eager(monkeypatch):
    steps = 9
    l_g, p_g, b_g, o_g, replays = _run("1", steps, monkeypatch)
    l_e, p_e, b_e, o_e, replays_e = _run("0", steps, monkeypatch)
    assert replays_e == 0
    # AFTER (2) eager steps, then graphed; the short batch and nothing else eager
    assert replays == steps - 2 - 1
    assert l_g == l_e
    assert torch.equal(p_g, p_e)
    assert torch.equal(b_g, b_e)              # BN running statistics: warm-up side effects undone
    assert all(torch.equal(a, b) for a, b in zip(o_g, o_e))  # num_batches_tracked


def test_graphed_engine_with_side_stream_reference(monkeypatch):
    """graphed (single-stream) vs the default eager engine (weight gradients on the side stream,
    a different split-K grid): same training within bf16 reduction-order noise"""
    from mi355x_dp.parallel import step_graph
    l_g, p_g, *_ = _run("1", 6, monkeypatch, wgrad_stream=True)
    monkeypatch.setattr(step_graph, "MODE", "0")
    from mi355x_dp.models import get_model
    from mi355x_dp.parallel import DataParallel
    torch.manual_seed(0)
    eng = DataParallel(get_model("resnet18", num_classes=1000).cuda(), foreign_optimizer=True)
    opt = torch.optim.SGD(eng.parameters(), lr=0.01, momentum=0.9)
    crit = torch.nn.CrossEntropyLoss().cuda()
    g = torch.Generator().manual_seed(5)
    for i in range(6):
        n = 32 if i != 4 else 10
        data = torch.randn(n, 3, 32, 32, generator=g).cuda()
        target = torch.randint(0, 10, (n,), generator=g).cuda()
        opt.zero_grad()
        loss = crit(eng(data), target)
        loss.backward()
        opt.step()
        if i == 4:
            eng.eval()
            with torch.no_grad():
                eng(torch.randn(100, 3, 32, 32, generator=g).cuda())
            eng.train()
    torch.cuda.synchronize()
    assert float(loss) == pytest.approx(l_g[-1], rel=2e-2)
    d = (eng.flat.data - p_g).abs().max()
    assert float(d) < 1e-3


@pytest.mark.parametrize("backend", ["nccl", "smddp"])
def test_graphed_comm_modes_match_eager(backend):
    """a replayed backward's bucket collectives captured INTO the graph (default
    for RCCL paths), behind gates enqueued before the replay, or launched after it -- every mode
    equals the eager engine bit for bit at world 1 with every collective issued (force_comm),
    and the captured mode issues no per-step collective from the host"""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "graphed_capture_check.py"), "--backend", backend],
                       capture_output=True, text=True, timeout=300, cwd=root,
                       env={**os.environ, "MASTER_PORT": str(29593 + (backend == "smddp"))})
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    steps = len(out["eager_losses"])
    for mode in ("capture", "gates", "after"):
        m = out[mode]
        # gates need a high-priority stream of their own (step_graph.gates_stream_high_priority):
        # torch nccl's normal-priority comm stream would wait on them, so a gates request resolves
        # to "after" there
        want = "after" if (mode == "gates" and backend == "nccl") else mode
        assert m["modes"] == [want], (mode, m)
        assert m["replays"] == steps - 2 - 1, (mode, m)
        assert m["losses_equal"] and m["params_equal"] and m["buffers_equal"], (mode, m)
    # captured: the replays' collectives come from the graph, not from the host reducer
    assert out["capture"]["comm_calls"] < out["gates"]["comm_calls"] == out["eager_comm_calls"], out
