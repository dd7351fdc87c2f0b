"""IPC mesh collectives at world size W (IPC-only smddp; ranks may share one GPU): reduce-scatter
(fp32 SUM / AVG, bf16, in place, chunked past the slot), all-gather (fp32, bf16, odd bytes) and the
chunked two-shot all-reduce against exact references, also with rank 0's tensors misaligned.  Prints MESH_OK <rank> <world>."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.append(os.path.join(ROOT, "compat"))
import smdistributed.dataparallel.torch.torch_smddp  # noqa: E402,F401

dist.init_process_group(backend="smddp")
r, w = dist.get_rank(), dist.get_world_size()
tot = sum(q + 1 for q in range(w))
for S in (1, 1000, 300_001):
    base = torch.arange(w * S, device="cuda", dtype=torch.float32)
    for op in (dist.ReduceOp.SUM, dist.ReduceOp.AVG):
        out = torch.empty(S, device="cuda")
        dist.reduce_scatter_tensor(out, base * (r + 1), op=op)
        ref = base[r * S:(r + 1) * S] * tot / (w if op == dist.ReduceOp.AVG else 1)
        assert torch.allclose(out, ref, rtol=1e-6), (S, op, (out - ref).abs().max().item())
    x = base * (r + 1)
    dist.reduce_scatter_tensor(x[r * S:(r + 1) * S], x)
    assert torch.allclose(x[r * S:(r + 1) * S], base[r * S:(r + 1) * S] * tot, rtol=1e-6)
    h = torch.full((w * S,), 0.5 + r, device="cuda", dtype=torch.bfloat16)
    ho = torch.empty(S, device="cuda", dtype=torch.bfloat16)
    dist.reduce_scatter_tensor(ho, h)
    want = sum(0.5 + q for q in range(w))
    assert float(ho.float().min()) == want and float(ho.float().max()) == want
    g = torch.zeros(w * S, device="cuda")
    g[r * S:(r + 1) * S] = base[r * S:(r + 1) * S] + 0.5
    dist.all_gather_into_tensor(g, g[r * S:(r + 1) * S])
    assert torch.equal(g, base + 0.5)
    t = torch.arange(S, device="cuda", dtype=torch.float32) * (r + 1)
    dist.all_reduce(t)
    assert torch.allclose(t, torch.arange(S, device="cuda", dtype=torch.float32) * tot, rtol=1e-6)
# rank-local misalignment: rank 0's tensors sit 4 bytes past a 16-byte boundary, the
# others' are aligned -- every rank must still cut each payload into the same per-block pieces
off = 1 if r == 0 else 0
for S in (5, 1000, 65_537, 300_001):
    buf = torch.zeros(w * S + 8, device="cuda")
    t = buf[off:off + S]
    t.copy_(torch.arange(S, device="cuda", dtype=torch.float32) * (r + 1))
    dist.all_reduce(t)
    assert torch.allclose(t, torch.arange(S, device="cuda", dtype=torch.float32) * tot, rtol=1e-6), S
    x = buf[off:off + w * S]
    x.copy_(torch.arange(w * S, device="cuda", dtype=torch.float32) * (r + 1))
    o = torch.zeros(S + 8, device="cuda")[off:off + S]
    dist.reduce_scatter_tensor(o, x)
    assert torch.allclose(o, torch.arange(r * S, (r + 1) * S, device="cuda", dtype=torch.float32) * tot, rtol=1e-6), S
    g = buf[off:off + w * S]
    g.zero_()
    g[r * S:(r + 1) * S] = torch.arange(r * S, (r + 1) * S, device="cuda", dtype=torch.float32)
    dist.all_gather_into_tensor(g, g[r * S:(r + 1) * S].clone())
    assert torch.equal(g, torch.arange(w * S, device="cuda", dtype=torch.float32)), S
    b = buf[off:off + S]
    b.fill_(float(r))
    dist.broadcast(b, 0)
    assert float(b.min()) == 0 and float(b.max()) == 0, S
    hb = torch.zeros(w * S + 8, device="cuda", dtype=torch.bfloat16)[off:off + w * S]
    hb.fill_(0.5 + r)
    ho = torch.zeros(S + 8, device="cuda", dtype=torch.bfloat16)[off:off + S]
    dist.reduce_scatter_tensor(ho, hb)
    assert float(ho.float().min()) == want and float(ho.float().max()) == want, S
u = torch.empty(w * 3, device="cuda", dtype=torch.uint8)
dist.all_gather_into_tensor(u, torch.full((3,), 7 + r, device="cuda", dtype=torch.uint8))
assert u.tolist() == sum(([7 + q] * 3 for q in range(w)), []), u.tolist()
# broadcast and MAX (the generic one-shot), then the per-size path probe (IPC one-shot vs two-shot;
# an IPC-only backend has no RCCL to compare with) and the flag memory kind
b = torch.full((1001,), float(r), device="cuda")
dist.broadcast(b, w - 1)
assert float(b.min()) == w - 1 and float(b.max()) == w - 1
m = torch.tensor([float(r)], device="cuda", dtype=torch.float64)
dist.all_reduce(m, op=dist.ReduceOp.MAX)
assert float(m) == w - 1
from mi355x_dp.parallel import comm_paths  # noqa: E402
info = comm_paths.ipc_info()
assert info["on"] == 1 and info["only"] == 1, info
rows = comm_paths.probe_paths(sizes_mb=(0.0625, 0.5), iters=2, warmup=1)
assert all(x["ipc_oneshot"] > 0 and x["ipc_twoshot"] > 0 and x["rccl"] < 0 for x in rows), rows
thr, one = comm_paths.choose_paths(rows)
t = torch.arange(4096, device="cuda", dtype=torch.float32) * (r + 1)
dist.all_reduce(t)  # thresholds restored after the probe: still exact
assert torch.allclose(t, torch.arange(4096, device="cuda", dtype=torch.float32) * tot, rtol=1e-6)
torch.cuda.synchronize()
flags = "uncached" if info["flags_uncached"] else "finegrained" if info["flags_finegrained"] else "coarse"
print("MESH_OK", r, w, "flags", flags, "rows", rows, flush=True)
dist.destroy_process_group()
