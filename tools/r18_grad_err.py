"""Per-parameter gradient error of the native ResNet-18 bf16 step vs fp32 PyTorch, next to stock
bf16 (MIOpen) on the same problem (worst margin over parameters, 3 seeds)."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch, torch.nn.functional as F
from tests.test_kernels_gpu import rel_err, rel_l2
from mi355x_dp.models import resnet18
from mi355x_dp.models.stock import stock_resnet
from mi355x_dp.ops import cross_entropy
BF=torch.bfloat16; CL=torch.channels_last
worst=[]
for seed in range(3):
    torch.manual_seed(seed)
    m = resnet18(num_classes=10).cuda()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.randn(8, 3, 64, 64, device="cuda"); y = torch.randint(0, 10, (8,), device="cuda")
    cross_entropy(m(x), y).backward()
    ref = stock_resnet("resnet18", 10).cuda(); ref.load_state_dict(sd)
    F.cross_entropy(ref(x), y).backward()
    st = stock_resnet("resnet18", 10).cuda().to(BF).to(memory_format=CL); st.load_state_dict(sd)
    F.cross_entropy(st(x.to(BF).contiguous(memory_format=CL)).float(), y).backward()
    pn, pr, ps = dict(m.named_parameters()), dict(ref.named_parameters()), dict(st.named_parameters())
    r = max(((rel_err(pn[n].grad, pr[n].grad) - 1.5*rel_err(ps[n].grad, pr[n].grad), n, rel_err(pn[n].grad, pr[n].grad), rel_err(ps[n].grad, pr[n].grad)) for n in pr))
    print(os.environ.get("MI355X_DP_KERNEL_VARIANT",""), seed, "worst margin (max-abs)", r)
    r = max(((rel_l2(pn[n].grad, pr[n].grad) - 1.5*rel_l2(ps[n].grad, pr[n].grad), n, rel_l2(pn[n].grad, pr[n].grad), rel_l2(ps[n].grad, pr[n].grad)) for n in pr))
    print(os.environ.get("MI355X_DP_KERNEL_VARIANT",""), seed, "worst margin (l2)", r)
