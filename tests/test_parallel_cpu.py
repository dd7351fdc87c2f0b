"""Distributed semantics on CPU with gloo, world_size 2: the flat-buffer bucketed
engine equals single-process full-batch SGD, replicas stay bit-identical, the smddp backend name
works (gloo fallback on hosts without a GPU), and the reference's manual _average_gradients on
top of DDP is a numerical no-op (C42)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    if backend == "smddp":
        sys.path.append(os.path.join(ROOT, "compat"))
        import smdistributed.dataparallel.torch.torch_smddp  # noqa: F401
    dist.init_process_group(backend, rank=rank, world_size=world)


def _model():
    from mi355x_dp.models import Net
    torch.manual_seed(0)
    return Net()


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(16, 3, 32, 32, generator=g), torch.randint(0, 10, (16,), generator=g)


def _worker_engine(rank, world, port, q, backend):
    try:
        _worker_engine_body(rank, world, port, q, backend)
    except Exception as e:  # surface worker failures instead of timing out
        q.put((rank, e, -1, -1))
        raise


def _worker_engine_body(rank, world, port, q, backend):
    _init(rank, world, port, backend)
    from mi355x_dp.parallel import DataParallel, FlatSGD
    m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01)
    opt = FlatSGD(m, lr=0.1, momentum=0.9, weight_decay=1e-3)
    x, y = _data()
    shard = slice(rank * 8, (rank + 1) * 8)
    for _ in range(3):
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x[shard]), y[shard]).backward()
        opt.step()
    q.put((rank, m.flat.data.clone().numpy(), len(m.buckets), m.comm_calls))  # by value: the child may exit first
    dist.destroy_process_group()


@pytest.mark.parametrize("backend", ["gloo", "smddp"])
def test_engine_matches_single_process(backend):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_engine, args=(r, 2, port, q, backend)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (torch.from_numpy(d) if not isinstance(d, Exception) else d, nb, nc))
               for r, d, nb, nc in [q.get(timeout=120) for _ in ps])
    for p in ps:
        p.join(60)
    for r, (d, _, _) in res.items():
        assert not isinstance(d, Exception), f"rank {r}: {d!r}"
    assert res[0][1] > 1, "expected several buckets"
    assert torch.equal(res[0][0], res[1][0]), "replicas diverged"
    # reference: one process, full batch, torch.optim.SGD
    m = _model()
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-3)
    x, y = _data()
    for _ in range(3):
        opt.zero_grad()
        # mean of the two shard losses == DDP average of shard gradients
        (0.5 * (torch.nn.functional.cross_entropy(m(x[:8]), y[:8]) +
                torch.nn.functional.cross_entropy(m(x[8:]), y[8:]))).backward()
        opt.step()
    from mi355x_dp.parallel import FlatParams
    ref = FlatParams(list(reversed(list(m.parameters()))), bf16_copy=False, kernel_layout_ids=set()).data
    assert torch.allclose(res[0][0], ref, atol=1e-5, rtol=1e-4)


def _worker_manual_avg(rank, world, port, q):
    _init(rank, world, port)
    torch.manual_seed(0)
    m = torch.nn.parallel.DistributedDataParallel(_model())
    x, y = _data()
    torch.nn.functional.cross_entropy(m(x[rank * 8:(rank + 1) * 8]), y[rank * 8:(rank + 1) * 8]).backward()
    before = [p.grad.clone() for p in m.parameters()]
    size = float(dist.get_world_size())  # reference cpu.py:87-92 on top of DDP
    for p in m.parameters():
        dist.all_reduce(p.grad.data, op=dist.ReduceOp.SUM)
        p.grad.data /= size
    after = [p.grad for p in m.parameters()]
    q.put(max(float((a - b).abs().max()) for a, b in zip(after, before)))
    dist.destroy_process_group()


def test_manual_average_on_top_of_ddp_is_noop():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_manual_avg, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    diffs = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(60)
    assert max(diffs) < 1e-6


def test_bucket_plan():
    from mi355x_dp.parallel import plan_buckets
    b = plan_buckets([4, 4, 4, 100, 4, 4], cap_bytes=10, first_cap_bytes=8)
    assert b == [[0, 1], [2], [3], [4, 5]]
    assert sum(len(x) for x in b) == 6


def test_flat_params_layout_and_state_dict():
    from mi355x_dp.models import resnet18
    from mi355x_dp.parallel import DataParallel
    m = resnet18()
    ref = {k: v.clone() for k, v in m.state_dict().items()}
    e = DataParallel(m)
    sd = e.state_dict()
    assert list(sd.keys())[0] == "module.conv1.weight"
    for k, v in ref.items():
        assert torch.equal(sd["module." + k], v)
        assert sd["module." + k].is_contiguous()
    # conv weights live in the flat buffer in [K][R][S][C] (channels_last) order
    w = m.layer1[0].conv1.weight
    assert w.is_contiguous(memory_format=torch.channels_last)
    assert w.data_ptr() >= e.flat.data.data_ptr()
    assert w.grad is not None and w.grad.data_ptr() >= e.flat.grad.data_ptr()


def test_native_reducer_planner():
    from mi355x_dp.parallel import _reducer_native
    ext = _reducer_native.load()
    if ext is None:
        pytest.skip("native reducer not built")
    sizes = [4] * 10 + [100] + [4] * 5
    b = ext.plan_buckets(sizes, 16, 8, 12)
    flat = [i for bb in b for i in bb]
    assert flat == list(range(len(sizes)))            # contiguous, in order, complete
    assert sum(sizes[i] for i in b[0]) <= 8            # small first bucket
    assert sum(sizes[i] for i in b[-1]) <= 12          # small last (exposed-tail) bucket
    # link-aware cap grows with world size (more rings over more links), clamped
    caps = [ext.link_aware_cap(w) for w in (2, 4, 8)]
    assert caps[0] <= caps[1] <= caps[2] <= 64 << 20 and caps[0] >= 4 << 20


def _worker_reducer(rank, world, port, q, py):
    try:
        if py:
            os.environ["MI355X_DP_PY_REDUCER"] = "1"
        _init(rank, world, port)
        from mi355x_dp.parallel import DataParallel, FlatSGD
        m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01)
        opt = FlatSGD(m, lr=0.05, momentum=0.9)
        x, y = _data()
        shard = slice(rank * 8, (rank + 1) * 8)
        for _ in range(2):
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x[shard]), y[shard]).backward()
            opt.step()
        q.put((rank, m.native_reducer, m.flat.data.clone().numpy(), m.comm_calls))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e, None, -1))
        raise


def test_native_reducer_matches_python_reducer():
    from mi355x_dp.parallel import _reducer_native
    if _reducer_native.load() is None:
        pytest.skip("native reducer not built")
    out = {}
    for py in (False, True):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_worker_reducer, args=(r, 2, port, q, py)) for r in range(2)]
        for p in ps:
            p.start()
        res = [q.get(timeout=120) for _ in ps]
        for p in ps:
            p.join(60)
        for r, native, d, calls in res:
            assert not isinstance(native, Exception), repr(native)
            assert native is (not py)
            assert calls > 2
        out[py] = res[0][2]
    assert (out[False] == out[True]).all()
