"""Debug: run the all-reduce (A) and balanced-shard (B) engines twice each, sequentially, on 2
IPC-only ranks sharing one GPU; print per-step losses and shadow consistency."""
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
from mi355x_dp.models import resnet18  # noqa: E402
from mi355x_dp.ops import cross_entropy  # noqa: E402
from mi355x_dp.parallel import DataParallel, FlatSGD  # noqa: E402

mode_list = os.environ.get("MODES", "A,A,B,B").split(",")
for tag in mode_list:
    shard = tag == "B"
    torch.manual_seed(0)
    e = DataParallel(resnet18(num_classes=10).cuda(), bucket_cap_mb=8, min_bucket_mb=0, shard_optimizer=shard)
    opt = FlatSGD(e, lr=0.05, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device="cuda").manual_seed(r)
    losses = []
    for step in range(3):
        x = torch.randn(16, 3, 32, 32, device="cuda", generator=g)
        y = torch.randint(0, 10, (16,), device="cuda", generator=g)
        e.zero_grad()
        loss = cross_entropy(e(x), y)
        loss.backward()
        opt.step()
        e.wait_param_sync()
        torch.cuda.synchronize()
        sh = (e.flat.bf16.float() - e.flat.data.to(torch.bfloat16).float()).abs().max().item()
        losses.append(round(float(loss), 6))
        gs = float(e.flat.grad.double().abs().sum())
        print(f"rank {r} {tag} step {step} loss {losses[-1]} shadow_err {sh} |g|1 {gs:.6e} "
              f"|p|1 {float(e.flat.data.double().abs().sum()):.9e}", flush=True)
    del e, opt
dist.destroy_process_group()
