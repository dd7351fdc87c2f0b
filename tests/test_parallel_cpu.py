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
    m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0)
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
    # on host tensors the engine keeps torch's layout (stock CPU convolutions round the same); the
    # native kernels' [K][R][S][C] (channels_last) order is used for GPU engines / kernel_layout_ids
    w = m.layer1[0].conv1.weight
    assert w.is_contiguous()
    assert w.data_ptr() >= e.flat.data.data_ptr()
    from mi355x_dp.parallel.flat import FlatParams
    m2 = resnet18()
    FlatParams(list(m2.parameters()), bf16_copy=False, kernel_layout_ids={id(m2.layer1[0].conv1.weight)})
    assert m2.layer1[0].conv1.weight.is_contiguous(memory_format=torch.channels_last)
    assert m2.layer1[0].conv2.weight.is_contiguous()
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
        m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0)
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


def test_planner_merges_small_buckets():
    """No latency-only sliver buckets (the lone 4 KB fc.bias first bucket): every
    planned bucket is >= min_bytes unless it is the only one; native == Python planner; a first
    bucket capped below the first big tensor takes that tensor."""
    from mi355x_dp.parallel import _reducer_native
    from mi355x_dp.parallel.ddp import plan_buckets
    from mi355x_dp.models import get_model
    ext = _reducer_native.load()
    for name in ("resnet18", "resnet50", "vit_b_16"):
        ps = list(reversed([p for p in get_model(name).parameters() if p.requires_grad]))
        sizes = [p.numel() * 4 for p in ps]
        cap, first, last, mn = 32 << 20, 2 << 20, 4 << 20, 1 << 20
        plan = plan_buckets(sizes, cap, first, last, mn)
        assert [i for b in plan for i in b] == list(range(len(sizes)))
        bsz = [sum(sizes[i] for i in b) for b in plan]
        assert len(plan) == 1 or min(bsz) >= mn, (name, bsz)
        assert max(bsz) <= cap + max(sizes), (name, bsz)
        if ext is not None:
            assert [list(b) for b in ext.plan_buckets(sizes, cap, first, last, mn)] == plan
    # resnet50: fc.bias (4 KB) + fc.weight (8 MB) form the first bucket
    ps = list(reversed([n for n, p in get_model("resnet50").named_parameters()]))
    plan = plan_buckets([p.numel() * 4 for p in reversed(list(get_model("resnet50").parameters()))],
                        32 << 20, 2 << 20, 4 << 20, 1 << 20)
    assert [ps[i] for i in plan[0]] == ["fc.bias", "fc.weight"]
    assert merge_ok([[0], [1, 2], [3]], [10, 1, 1, 10], 5) == [[0], [1, 2, 3]]
    assert merge_ok([[0], [1], [2]], [10, 10, 1], 5) == [[0], [1, 2]]


def merge_ok(b, sizes, mn):
    from mi355x_dp.parallel.ddp import merge_small_buckets
    return merge_small_buckets(b, sizes, mn)


def test_stream_order_checker_cpu():
    """check_stream_order=True: a normal step passes and yields the same gradients as the plain
    path; a gradient changed after its bucket was handed to the collective is reported."""
    from mi355x_dp.parallel import DataParallel
    from mi355x_dp.parallel.health import StreamOrderViolation
    x, y = _data()
    grads = {}
    for check in (False, True):
        e = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0,
                         check_stream_order=check)
        assert e.reducer is None or not check
        e.zero_grad()
        torch.nn.functional.cross_entropy(e(x), y).backward()
        e.finish_gradient_sync()
        grads[check] = e.flat.grad.clone()
        assert e.order_violations == []
    assert torch.equal(grads[False], grads[True])
    # a "producer" that writes after the grad-ready signal: mark ready, then modify the slice
    e = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0, check_stream_order=True)
    e.zero_grad()
    e._reset()
    for i in e.buckets[0]:
        e._mark_ready(i)
    lo, hi = e.bucket_ranges[0]
    e.flat.grad[lo:hi] += 1.0  # late write
    with pytest.raises(StreamOrderViolation, match="bucket 0"):
        e.finish_gradient_sync()


def _worker_force_comm(q, port):
    try:
        _init(0, 1, port)
        from mi355x_dp.parallel import DataParallel, FlatSGD
        m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0, force_comm=True)
        opt = FlatSGD(m, lr=0.05, momentum=0.9)
        x, y = _data()
        opt.zero_grad()
        torch.nn.functional.cross_entropy(m(x), y).backward()
        opt.step()
        q.put((len(m.buckets), m.comm_calls, [t[0] for t in m.bucket_trace]))
        dist.destroy_process_group()
    except Exception as e:
        q.put(e)
        raise


def test_force_comm_world1():
    """force_comm issues every bucket collective at world size 1 (the comm path a one-GPU box can
    trace); the native reducer records the launch order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_force_comm, args=(q, _port()))
    p.start()
    r = q.get(timeout=120)
    p.join(60)
    assert not isinstance(r, Exception), repr(r)
    nb, calls, trace = r
    assert nb > 1 and calls == nb
    from mi355x_dp.parallel import _reducer_native
    if _reducer_native.load() is not None:
        assert trace[:nb] == list(range(nb)) and trace[-1] == -1


class _BNNet(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.c = torch.nn.Conv2d(3, 8, 3)
        self.bn = torch.nn.BatchNorm2d(8)
        self.fc = torch.nn.Linear(8, 10)

    def forward(self, x):
        return self.fc(torch.relu(self.bn(self.c(x))).mean((2, 3)))


def _worker_buffers(rank, world, port, q):
    try:
        _init(rank, world, port)
        from mi355x_dp.parallel import DataParallel, FlatSGD
        torch.manual_seed(0)
        m = DataParallel(_BNNet(), min_bucket_mb=0)
        opt = FlatSGD(m, lr=0.05, momentum=0.9)
        x, y = _data()
        shard = slice(rank * 8, (rank + 1) * 8)
        seen = []
        for _ in range(3):
            opt.zero_grad()
            out = m(x[shard] * (1 + rank))  # different batch statistics per rank
            torch.nn.functional.cross_entropy(out, y[shard]).backward()
            opt.step()
            seen.append(m.module.bn.running_mean.clone().numpy())
        q.put((rank, seen, int(m.module.bn.num_batches_tracked)))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e, None))
        raise


def test_buffer_broadcast_async():
    """BN buffers are broadcast from rank 0 asynchronously behind backward (not before every
    forward): after each optimizer step every rank holds rank 0's post-forward running stats."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_buffers, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (s, n) for r, s, n in [q.get(timeout=120) for _ in ps]}
    for p in ps:
        p.join(60)
    for r, (s, n) in res.items():
        assert not isinstance(s, Exception), repr(s)
        assert n == 3
    for a, b in zip(res[0][0], res[1][0]):
        assert (a == b).all()


def _worker_bf16_comm(rank, world, port, q, py, comm):
    try:
        if py:
            os.environ["MI355X_DP_PY_REDUCER"] = "1"
        _init(rank, world, port)
        from mi355x_dp.parallel import DataParallel, FlatSGD
        m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0, grad_comm=comm)
        opt = FlatSGD(m, lr=0.1, momentum=0.9)
        x, y = _data()
        shard = slice(rank * 8, (rank + 1) * 8)
        for _ in range(3):
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x[shard]), y[shard]).backward()
            opt.step()
        q.put((rank, m.flat.data.clone().numpy(), m.native_reducer, m.reducer.comm_bytes if m.reducer else -1))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e, None, None))
        raise


def test_bf16_gradient_allreduce():
    """grad_comm='bf16': buckets are exchanged as bf16 (half the bytes), summed identically on every
    rank (replicas bit-identical) and cast back into the fp32 gradient; the trajectory stays within
    bf16 rounding of the fp32 exchange.  Native and Python reducers agree."""
    out = {}
    for py, comm in ((False, "fp32"), (False, "bf16"), (True, "bf16")):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_worker_bf16_comm, args=(r, 2, port, q, py, comm)) for r in range(2)]
        for p in ps:
            p.start()
        res = {r: (d, nat, nb) for r, d, nat, nb in [q.get(timeout=120) for _ in ps]}
        for p in ps:
            p.join(60)
        for r, (d, nat, nb) in res.items():
            assert not isinstance(d, Exception), repr(d)
        assert (res[0][0] == res[1][0]).all(), (py, comm)
        out[(py, comm)] = res[0]
    f32, b16, b16py = out[(False, "fp32")], out[(False, "bf16")], out[(True, "bf16")]
    assert b16[1] is True and b16py[1] is False
    assert b16[2] * 2 == f32[2] > 0  # half the bytes on the wire
    assert (b16[0] == b16py[0]).all()
    assert abs(b16[0] - f32[0]).max() < 2e-3
    assert (b16[0] != f32[0]).any()  # the exchange really was rounded


def _big_model():
    torch.manual_seed(0)
    # ~12.6 M fp32 parameters (50 MB of gradient): the DEFAULT planner splits it into several buckets
    return torch.nn.Sequential(torch.nn.Linear(256, 4096), torch.nn.ReLU(), torch.nn.Linear(4096, 2048),
                               torch.nn.ReLU(), torch.nn.Linear(2048, 1024), torch.nn.ReLU(),
                               torch.nn.Linear(1024, 10))


def _worker_default_plan(rank, world, port, q):
    try:
        _init(rank, world, port)
        from mi355x_dp.parallel import DataParallel, FlatSGD
        m = DataParallel(_big_model())  # default bucket plan (link-aware cap, min-size merge)
        opt = FlatSGD(m, lr=0.05, momentum=0.9)
        g = torch.Generator().manual_seed(10 + rank)
        for _ in range(3):
            x, y = torch.randn(32, 256, generator=g), torch.randint(0, 10, (32,), generator=g)
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            opt.step()
        q.put((rank, m.flat.data.clone().numpy(), [len(b) for b in m.buckets], m.comm_calls))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e, None, -1))
        raise


def test_four_ranks_default_plan():
    """4 gloo ranks with the default bucket planner (a 4-rank default-plan run had
    stalled on a GPU box -- root-caused to hardware-queue oversubscription of ranks sharing one GPU,
    profiles/multirank_rehearsal.md): every rank finishes, launches the same number of bucket
    collectives, and ends with bit-identical replicas."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_default_plan, args=(r, 4, port, q)) for r in range(4)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, d, plan, calls = q.get(timeout=240)
        res[r] = (d, plan, calls)
    for p in ps:
        p.join(60)
    for r, (d, _, _) in res.items():
        assert not isinstance(d, Exception), f"rank {r}: {d!r}"
    plans = {tuple(v[1]) for v in res.values()}
    assert len(plans) == 1 and len(next(iter(plans))) >= 2, plans
    assert len({v[2] for v in res.values()}) == 1
    for r in range(1, 4):
        assert (res[r][0] == res[0][0]).all(), f"rank {r} diverged"


def _worker_calibrate(rank, world, port, q):
    try:
        _init(rank, world, port)
        from mi355x_dp.parallel import DataParallel
        from mi355x_dp.parallel.ddp import calibrated_cap
        m = DataParallel(_big_model(), calibrate=True)
        c = m.calibration
        assert c is not None and c["alpha_us"] > 0 and c["algbw_GBps"] > 0
        assert int(c["cap_mb"] * 2**20) in range(4 << 20, (64 << 20) + 1)
        assert calibrated_cap(c["alpha_us"], c["algbw_GBps"]) >= 4 << 20
        q.put((rank, c, [len(b) for b in m.buckets]))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e, None))
        raise


def test_calibrated_bucket_plan_agrees_across_ranks():
    """DataParallel(calibrate=True): the all-reduce alpha-beta fit is reduced (MAX) over ranks, so
    every rank derives the same bucket cap and plan (a rank-dependent plan would deadlock)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_calibrate, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (c, plan)) for r, c, plan in [q.get(timeout=180) for _ in ps])
    for p in ps:
        p.join(60)
    for r, (c, _) in res.items():
        assert not isinstance(c, Exception), f"rank {r}: {c!r}"
    assert res[0] == res[1]


def _worker_shard(rank, world, port, q, py, shard, comm):
    try:
        if py:
            os.environ["MI355X_DP_PY_REDUCER"] = "1"
        _init(rank, world, port)
        from mi355x_dp.parallel import DataParallel, FlatSGD
        m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0, grad_comm=comm,
                         shard_optimizer=shard)
        opt = FlatSGD(m, lr=0.1, momentum=0.9, weight_decay=1e-3)
        x, y = _data()
        per = 16 // world
        part = slice(rank * per, (rank + 1) * per)
        for _ in range(3):
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x[part]), y[part]).backward()
            opt.step()
        sd = m.state_dict()  # joins the parameter all-gathers
        osd = opt.state_dict()
        ranges = [(lo, hi) for lo, hi in m.bucket_ranges]
        q.put((rank, {k: v.clone().numpy() for k, v in sd.items()}, m.native_reducer, m.comm_calls,
               osd["momentum_buf"].numel(), m.flat.numel, ranges, osd.get("shard")))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e, None, None, None, None, None, None))
        raise


def _run_shard(world, py, shard, comm="fp32"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_shard, args=(r, world, port, q, py, shard, comm)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, *rest = q.get(timeout=180)
        res[r] = rest
    for p in ps:
        p.join(60)
    for r, v in res.items():
        assert not isinstance(v[0], Exception), f"rank {r}: {v[0]!r}"
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_balanced_shard_optimizer_matches_allreduce(world):
    """shard_optimizer=True (SMDDP balanced shards: reduce-scatter, shard-local SGD, all-gather):
    every rank ends with the same parameters as the all-reduce engine, replicas bit-identical, each
    rank's momentum is 1/world of the (padded) flat buffer, every bucket splits into equal shards,
    and the native and Python reducers agree bit for bit."""
    ref = _run_shard(world, py=False, shard=False)
    nat = _run_shard(world, py=False, shard=True)
    pyr = _run_shard(world, py=True, shard=True)
    for res in (nat, pyr):
        for r in range(1, world):
            for k in res[0][0]:
                assert (res[r][0][k] == res[0][0][k]).all(), f"rank {r} diverged at {k}"
        for k, v in ref[0][0].items():
            assert abs(res[0][0][k] - v).max() < 1e-5, k
    assert nat[0][1] is True and pyr[0][1] is False
    for k in nat[0][0]:
        assert (nat[0][0][k] == pyr[0][0][k]).all(), k
    numel, ranges = nat[0][4], nat[0][5]
    assert all((hi - lo) % (64 * world) == 0 for lo, hi in ranges) and len(ranges) > 1
    assert nat[0][3] * world == numel  # packed momentum: this rank's shards only
    assert [{k: nat[r][6][k] for k in ("rank", "world")} for r in range(world)] == \
        [{"rank": r, "world": world} for r in range(world)]
    assert all(nat[r][6]["bucket_ranges"] == nat[0][6]["bucket_ranges"] for r in range(world))
    # one reduce-scatter + one all-gather per bucket per step
    assert nat[0][2] == pyr[0][2] == 3 * 2 * len(ranges)


def test_balanced_shard_with_bf16_gradients():
    """shard_optimizer + grad_comm='bf16': bf16 reduce-scatter, fp32 shard update, fp32 all-gather;
    replicas bit-identical and within bf16 rounding of the fp32 all-reduce trajectory."""
    ref = _run_shard(2, py=False, shard=False)
    res = _run_shard(2, py=False, shard=True, comm="bf16")
    for k in res[0][0]:
        assert (res[1][0][k] == res[0][0][k]).all(), k
        assert abs(res[0][0][k] - ref[0][0][k]).max() < 2e-3, k


def _worker_no_sync(rank, world, port, q, py):
    try:
        if py:
            os.environ["MI355X_DP_PY_REDUCER"] = "1"
        _init(rank, world, port)
        from mi355x_dp.parallel import DataParallel, FlatSGD
        m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0,
                         device_ids=None, find_unused_parameters=True, static_graph=True)
        opt = FlatSGD(m, lr=0.1, momentum=0.9)
        x, y = _data()
        part = slice(rank * 8, (rank + 1) * 8)
        calls = []
        for _ in range(2):
            opt.zero_grad()
            c0 = m.comm_calls
            with m.no_sync():  # first micro-batch: local accumulation only
                torch.nn.functional.cross_entropy(m(x[part][:4]), y[part][:4]).backward()
            calls.append(m.comm_calls - c0)
            torch.nn.functional.cross_entropy(m(x[part][4:]), y[part][4:]).backward()
            opt.step()
        q.put((rank, m.flat.data.clone().numpy(), calls, m.native_reducer))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e, None, None))
        raise


@pytest.mark.parametrize("py", [False, True])
def test_no_sync_gradient_accumulation(py):
    """DataParallel.no_sync() (torch DDP's accumulation API, with DDP's constructor kwargs): the
    micro-batch inside it issues no collective, the next backward reduces the accumulated sum, and
    the result equals one process accumulating all four micro-batch gradients."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_no_sync, args=(r, 2, port, q, py)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (d, c, nat) for r, d, c, nat in [q.get(timeout=120) for _ in ps]}
    for p in ps:
        p.join(60)
    for r, (d, _, _) in res.items():
        assert not isinstance(d, Exception), f"rank {r}: {d!r}"
    assert res[0][1] == [0, 0] and res[0][2] is (not py)
    assert (res[0][0] == res[1][0]).all()
    m = _model()
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x, y = _data()
    for _ in range(2):
        opt.zero_grad()
        for r in range(2):  # DDP: sum of micro-batch losses per rank, averaged over ranks
            for sl in (slice(r * 8, r * 8 + 4), slice(r * 8 + 4, r * 8 + 8)):
                (0.5 * torch.nn.functional.cross_entropy(m(x[sl]), y[sl])).backward()
        opt.step()
    from mi355x_dp.parallel import FlatParams
    ref = FlatParams(list(reversed(list(m.parameters()))), bf16_copy=False, kernel_layout_ids=set()).data
    assert torch.allclose(torch.from_numpy(res[0][0]), ref, atol=1e-5, rtol=1e-4)


def test_ddp_kwargs_validation():
    from mi355x_dp.parallel import DataParallel
    with pytest.raises(ValueError):
        DataParallel(_model(), dim=1)


def _worker_shard_resume(rank, world, port, q, ckpt):
    try:
        _init(rank, world, port)
        from mi355x_dp.parallel import DataParallel, FlatSGD
        from mi355x_dp.utils import load_checkpoint, save_checkpoint
        x, y = _data()
        part = slice(rank * 8, (rank + 1) * 8)

        def engine():
            m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0,
                             shard_optimizer=True)
            return m, FlatSGD(m, lr=0.1, momentum=0.9, weight_decay=1e-3)

        def step(m, opt):
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x[part]), y[part]).backward()
            opt.step()
        m, opt = engine()
        for _ in range(2):
            step(m, opt)
        save_checkpoint(ckpt, m, opt, step=2)
        for _ in range(2):
            step(m, opt)
        a = {k: v.clone() for k, v in m.state_dict().items()}
        m2, opt2 = engine()
        for p in m2.module.parameters():  # resume must not depend on the fresh init
            p.data.add_(1.0)
        info = load_checkpoint(ckpt, m2, opt2)
        for _ in range(2):
            step(m2, opt2)
        b = m2.state_dict()
        diff = max(float((a[k] - b[k]).abs().max()) for k in a)
        q.put((rank, diff, info["step"], os.path.exists(f"{ckpt}.optim-rank{rank}-of-{world}")))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e, None, None))
        raise


def test_balanced_shard_checkpoint_resume(tmp_path):
    """Resumable checkpoint of a balanced-shard job: every rank writes its optimizer shard next to
    the rank-0 checkpoint; resuming on fresh engines continues the exact trajectory."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ckpt = str(tmp_path / "ckpt.pt")
    ps = [ctx.Process(target=_worker_shard_resume, args=(r, 2, port, q, ckpt)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (d, s, e) for r, d, s, e in [q.get(timeout=120) for _ in ps]}
    for p in ps:
        p.join(60)
    for r, (d, s, e) in res.items():
        assert not isinstance(d, Exception), f"rank {r}: {d!r}"
        assert d == 0.0 and s == 2 and e, (r, d, s, e)


def _worker_comm_hook(rank, world, port, q, which):
    try:
        _init(rank, world, port)
        from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
        from mi355x_dp.parallel import DataParallel, FlatSGD
        m = DataParallel(_model(), bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0)
        if which == "allreduce":
            m.register_comm_hook(None, default_hooks.allreduce_hook)
        elif which == "fp16":
            m.register_comm_hook(None, default_hooks.fp16_compress_hook)
        seen = []
        if which == "custom":
            def hook(state, bucket):  # records the bucket interface, then a plain averaged all-reduce
                seen.append((bucket.index(), bucket.is_last(), len(bucket.parameters()),
                             sum(g.numel() for g in bucket.gradients()) <= bucket.buffer().numel()))
                t = bucket.buffer().div_(world)
                return dist.all_reduce(t, async_op=True).get_future().then(lambda f: f.value()[0])
            m.register_comm_hook("state", hook)
        opt = FlatSGD(m, lr=0.1, momentum=0.9)
        x, y = _data()
        part = slice(rank * 8, (rank + 1) * 8)
        for _ in range(3):
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x[part]), y[part]).backward()
            opt.step()
        q.put((rank, m.flat.data.clone().numpy(), seen, len(m.buckets)))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e, None, None))
        raise


def test_ddp_comm_hooks():
    """register_comm_hook with torch's own DDP hooks (allreduce_hook, fp16_compress_hook) and a
    custom hook: same trajectory as the engine's fused all-reduce (fp16: within fp16 rounding),
    replicas identical, GradBucket interface (index / is_last / parameters / gradients / buffer)."""
    out = {}
    for which in ("none", "allreduce", "fp16", "custom"):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_worker_comm_hook, args=(r, 2, port, q, which)) for r in range(2)]
        for p in ps:
            p.start()
        res = {r: (d, seen, nb) for r, d, seen, nb in [q.get(timeout=120) for _ in ps]}
        for p in ps:
            p.join(60)
        for r, (d, _, _) in res.items():
            assert not isinstance(d, Exception), f"{which} rank {r}: {d!r}"
        assert (res[0][0] == res[1][0]).all(), which
        out[which] = res[0]
    base = out["none"][0]
    assert abs(out["allreduce"][0] - base).max() < 1e-6
    assert abs(out["custom"][0] - base).max() < 1e-6
    assert 0 < abs(out["fp16"][0] - base).max() < 1e-2
    seen, nb = out["custom"][1], out["custom"][2]
    assert [s[0] for s in seen] == list(range(nb)) * 3
    assert [s[1] for s in seen[:nb]] == [False] * (nb - 1) + [True]
    assert all(s[2] > 0 and s[3] for s in seen)


def _worker_probe(rank, world, port, q):
    try:
        _init(rank, world, port)
        from mi355x_dp.parallel.ddp import probe_collectives
        q.put((rank, probe_collectives(sizes_mb=(0.25, 4.0), iters=2, warmup=1)))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, e))
        raise


def test_probe_collectives_agrees_across_ranks():
    """bench.py's post-timing fabric probe: all-reduce and RS+AG times, MAX over ranks (identical
    on every rank), positive bus bandwidths."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_probe, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    for r, v in res.items():
        assert not isinstance(v, Exception), f"rank {r}: {v!r}"
    assert res[0] == res[1] and len(res[0]) == 2
    assert res[0][0]["allreduce_ms"] > 0 and res[0][0]["allreduce_busbw_GBps"] >= 0 and "rs_plus_ag_ms" not in res[0][0]
    assert res[0][1]["rs_plus_ag_ms"] > 0 and res[0][1]["allreduce_bf16_same_elems_ms"] > 0


def test_shard_checkpoint_rejects_a_different_bucket_plan():
    """A balanced-shard optimizer checkpoint records the bucket plan its packed momentum was laid out
    for; loading it into an engine planned differently (other bucket caps) raises instead of pairing
    momentum with the wrong parameters -- even when the packed lengths happen to agree."""
    from mi355x_dp.parallel import DataParallel, FlatSGD
    e1 = DataParallel(_model(), shard_optimizer=True, bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0)
    o1 = FlatSGD(e1, lr=0.1, momentum=0.9)
    x, y = _data()
    torch.nn.functional.cross_entropy(e1(x), y).backward()
    o1.step()
    sd = o1.state_dict()
    assert sd["shard"]["bucket_ranges"] == [list(r) for r in e1.bucket_ranges]
    same = DataParallel(_model(), shard_optimizer=True, bucket_cap_mb=0.05, first_bucket_mb=0.01, min_bucket_mb=0)
    o_same = FlatSGD(same, lr=0.1, momentum=0.9)
    o_same.load_state_dict(sd)
    assert torch.equal(o_same.momentum_buf, o1.momentum_buf)
    other = DataParallel(_model(), shard_optimizer=True, bucket_cap_mb=0.2, first_bucket_mb=0.05, min_bucket_mb=0)
    assert len(other.buckets) != len(e1.buckets)
    with pytest.raises(ValueError, match="bucket plan"):
        FlatSGD(other, lr=0.1, momentum=0.9).load_state_dict(sd)


def _worker_engine_ddp(rank, world, port, q, use_engine):
    try:
        os.environ["MI355X_DP_ENGINE_DDP"] = "force" if use_engine else "0"
        _init(rank, world, port)
        from mi355x_dp.models import resnet18
        from mi355x_dp.parallel import engine_ddp
        engine_ddp.install()
        torch.manual_seed(0)
        model = resnet18(num_classes=10)
        # the reference's own calls (gpu.py:148, 156-168): stock class name, stock SGD, zero_grad
        ddp = torch.nn.parallel.DistributedDataParallel(model)
        # the unwrap idiom of scripts and libraries holds for the engine and the stock fallback
        assert isinstance(ddp, torch.nn.parallel.DistributedDataParallel), type(ddp)
        assert issubclass(type(ddp), torch.nn.parallel.DistributedDataParallel)
        opt = torch.optim.SGD(ddp.parameters(), lr=0.01, momentum=0.9)
        crit = torch.nn.CrossEntropyLoss()
        g = torch.Generator().manual_seed(7)
        x, y = torch.randn(8, 3, 32, 32, generator=g), torch.randint(0, 10, (8,), generator=g)
        part = slice(rank * 4, (rank + 1) * 4)
        grads = []
        for _ in range(3):
            opt.zero_grad()
            loss = crit(ddp(x[part]), y[part])
            loss.backward()
            grads.append(next(ddp.parameters()).grad.detach().clone())  # averaged when backward returns
            opt.step()
        ddp.eval()
        with torch.no_grad():
            ev = ddp(x[:2])
        sd = {k: v.detach().clone().numpy() for k, v in ddp.state_dict().items()}
        q.put((rank, type(ddp).__name__, sd, [g.numpy() for g in grads], ev.numpy()))
        dist.destroy_process_group()
        engine_ddp.uninstall()
    except Exception as e:
        import traceback
        traceback.print_exc()
        q.put((rank, e, None, None, None))


def test_engine_ddp_substitution_matches_stock_ddp():
    """The torch_smddp shim's engine-backed DistributedDataParallel (SURVEY §7.1 decision 2(b)):
    the reference's unmodified call sequence -- stock class name, stock optim.SGD with
    zero_grad(set_to_none), backward, step, eval forward, state_dict -- gives the same averaged
    gradients, parameters, BN buffers and module.-prefixed keys as torch's own DDP, on gloo world 2."""
    res = {}
    for use_engine in (True, False):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _port()
        ps = [ctx.Process(target=_worker_engine_ddp, args=(r, 2, port, q, use_engine)) for r in range(2)]
        for p in ps:
            p.start()
        out = {r: rest for r, *rest in [q.get(timeout=240) for _ in ps]}
        for p in ps:
            p.join(60)
        for r, (name, *_rest) in out.items():
            assert not isinstance(name, Exception), f"rank {r}: {name!r}"
        res[use_engine] = out
    assert res[True][0][0] == "DataParallel" and res[False][0][0] == "DistributedDataParallel"
    import numpy as np
    sd_e, sd_s = res[True][0][1], res[False][0][1]
    assert list(sd_e) == list(sd_s) and all(k.startswith("module.") for k in sd_e)
    # on host tensors the engine keeps torch's weight layout, so the math is the same op for op
    rel = lambda a, b: np.linalg.norm((a.astype(np.float64) - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-12)  # noqa
    for k in sd_s:
        if sd_s[k].dtype.kind == "f":
            assert rel(sd_e[k], sd_s[k].astype(np.float64)) < 1e-6, k
        else:
            assert np.array_equal(sd_e[k], sd_s[k]), k
    for ge, gs in zip(res[True][0][2], res[False][0][2]):
        assert rel(ge, gs.astype(np.float64)) < 1e-6
    assert rel(res[True][0][3], res[False][0][3].astype(np.float64)) < 1e-6
    # replicas identical on the engine path
    for k in sd_e:
        assert np.array_equal(res[True][0][1][k], res[True][1][1][k]), k


def test_engine_ddp_factory_class_semantics():
    """The installed factory behaves like torch's class for user code: subclassing the
    public name after the shim is imported yields a genuine subclass of torch's own DDP, and
    isinstance / issubclass accept the stock class and the engine."""
    from mi355x_dp.parallel import engine_ddp
    from mi355x_dp.parallel.ddp import DataParallel
    engine_ddp.install()
    try:
        import torch.nn.parallel as tnp
        stock = engine_ddp.stock_ddp()
        assert tnp.DistributedDataParallel is not stock

        class MyDDP(tnp.DistributedDataParallel):
            marker = 1

        assert issubclass(MyDDP, stock) and MyDDP.marker == 1 and MyDDP.__mro__[1] is stock
        assert issubclass(MyDDP, tnp.DistributedDataParallel)
        assert issubclass(DataParallel, tnp.DistributedDataParallel)
        assert not isinstance(torch.nn.Linear(2, 2), tnp.DistributedDataParallel)
        assert not issubclass(torch.nn.Linear, tnp.DistributedDataParallel)
    finally:
        engine_ddp.uninstall()


def test_comm_path_choice_from_probe_table():
    """smddp per-size path selection (parallel/comm_paths.py): IPC below the size where RCCL starts
    to win, one-shot below the size where the two-shot starts to win; unmeasured paths never
    chosen; a margin keeps near-ties on RCCL."""
    from mi355x_dp.parallel.comm_paths import choose_paths
    MB = 2**20
    rows = [
        {"bytes": MB // 4, "rccl": 0.060, "ipc_oneshot": 0.020, "ipc_twoshot": 0.030},
        {"bytes": 1 * MB, "rccl": 0.080, "ipc_oneshot": 0.050, "ipc_twoshot": 0.045},
        {"bytes": 4 * MB, "rccl": 0.110, "ipc_oneshot": 0.200, "ipc_twoshot": 0.090},
        {"bytes": 16 * MB, "rccl": 0.250, "ipc_oneshot": 0.800, "ipc_twoshot": 0.260},
        {"bytes": 32 * MB, "rccl": 0.420, "ipc_oneshot": 1.600, "ipc_twoshot": 0.400},
    ]
    assert choose_paths(rows) == (4 * MB, MB // 4)  # 16 MB: RCCL wins, so 32 MB stays RCCL too
    assert choose_paths(list(reversed(rows))) == (4 * MB, MB // 4)  # order-independent
    assert choose_paths(rows, margin=0.25) == (MB, MB // 4)  # 4 MB: 0.09 * 1.25 > 0.11
    # IPC not measured (or failed): RCCL everywhere
    assert choose_paths([{"bytes": MB, "rccl": 0.1, "ipc_oneshot": -1.0, "ipc_twoshot": None}]) == (0, 0)
    # RCCL not measured: IPC wins wherever it ran
    assert choose_paths([{"bytes": MB, "ipc_oneshot": 0.1, "ipc_twoshot": 0.2}]) == (MB, MB)


def test_wgrad_stream_auto_policy():
    """The weight-gradient side stream defaults on for BatchNorm conv nets and off for GEMM-bound
    models (ViT: its patch-embedding conv does not count)."""
    from mi355x_dp.models import get_model
    from mi355x_dp.parallel.ddp import _wgrad_stream_auto
    assert _wgrad_stream_auto(get_model("resnet50"))
    assert _wgrad_stream_auto(get_model("resnet18"))
    assert not _wgrad_stream_auto(get_model("vit_b_16"))


def _worker_capture_agree(rank, world, port, q, fail_rank):
    """rank ``fail_rank``'s graph capture raises; the others' would succeed (a fake that never gets
    to replay: the MIN agreement must disable graphs on every rank at the same step)."""
    try:
        _init(rank, world, port)
        from mi355x_dp.parallel import DataParallel, step_graph
        calls = {"capture": 0, "replay": 0}

        class FakeStep:
            comm_mode = "none"

            def __init__(self, engine, x):
                calls["capture"] += 1
                if rank == fail_rank:
                    raise RuntimeError("injected capture failure")

            def __call__(self, token, x):  # pragma: no cover - must never run
                calls["replay"] += 1
                raise AssertionError("replayed after a failed agreement")

            def busy(self):
                return False

        step_graph.eligible = lambda engine, args, kwargs: True
        step_graph.CapturedStep = FakeStep
        torch.manual_seed(0)
        ddp = DataParallel(_model(), foreign_optimizer=True)
        opt = torch.optim.SGD(ddp.parameters(), lr=0.05, momentum=0.9)
        x, y = _data()
        part = slice(rank * 8, (rank + 1) * 8)
        import warnings
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            for _ in range(step_graph.AFTER + 3):
                opt.zero_grad()
                torch.nn.functional.cross_entropy(ddp(x[part]), y[part]).backward()
                opt.step()
        msgs = [str(m.message) for m in w if "graph capture" in str(m.message)]
        q.put((rank, ddp.flat.data.clone().numpy(), calls, bool(ddp.__dict__.get("_graph_disabled")), msgs))
        dist.destroy_process_group()
    except Exception as e:
        import traceback
        traceback.print_exc()
        q.put((rank, e, None, None, None))


def test_graph_capture_agreement_is_rank_symmetric():
    """a capture that fails on rank 1 only must leave BOTH ranks eager (MIN
    all-reduce of the capture flag before any replay) -- no rank replays graphs while a peer runs
    eagerly, no hang, and the replicas stay bit-identical."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker_capture_agree, args=(r, 2, port, q, 1)) for r in range(2)]
    for p in ps:
        p.start()
    out = {r: rest for r, *rest in [q.get(timeout=120) for _ in ps]}
    for p in ps:
        p.join(60)
    for r, (d, *_rest) in out.items():
        assert not isinstance(d, Exception), f"rank {r}: {d!r}"
    for r in (0, 1):
        _d, calls, disabled, msgs = out[r]
        assert disabled, f"rank {r} kept graphs enabled"
        assert calls == {"capture": 1, "replay": 0}, (r, calls)
        assert msgs, f"rank {r} did not warn"
    assert "another rank" in out[0][3][0] and "injected" in out[1][3][0]
    assert torch.equal(torch.from_numpy(out[0][0]), torch.from_numpy(out[1][0])), "replicas diverged"


def test_graph_comm_mode_gates_need_high_priority(monkeypatch):
    """'gates' (queued before the replay) only on a high-priority gate / comm stream;
    torch nccl, or a normal-priority gate or smddp comm stream, falls back to 'after'."""
    from types import SimpleNamespace
    from mi355x_dp.parallel import step_graph
    eng = SimpleNamespace(comm_on=True, reducer=object(), _comm_hook=None)
    monkeypatch.setattr(step_graph, "capture_safe", lambda e: False)
    monkeypatch.setattr(step_graph, "GRAPH_COMM", "auto")
    for be, env, want in [("smddp", {}, "gates"), ("smddp", {"MI355X_DP_SMDDP_HIPRIO": "0"}, "after"),
                          ("smddp", {"MI355X_DP_GATE_PRIO": "0"}, "after"), ("nccl", {}, "after"),
                          ("gloo", {}, "gates")]:
        monkeypatch.setattr(step_graph, "_backend", lambda e, be=be: be)
        for k in ("MI355X_DP_SMDDP_HIPRIO", "MI355X_DP_GATE_PRIO"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        assert step_graph.comm_mode(eng) == want, (be, env)
    monkeypatch.setattr(step_graph, "capture_safe", lambda e: True)
    assert step_graph.comm_mode(eng) == "capture"
