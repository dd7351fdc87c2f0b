"""Per-block output difference, normalize-on-load on vs off (fused residual blocks)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mi355x_dp.ops.resblock as RB
from mi355x_dp.models import get_model

name, size, bs = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
if len(sys.argv) > 4:  # 0: the small-layer fused BN (statistics + apply in one launch) off
    from mi355x_dp.ops import _lib
    from mi355x_dp.ops import kernels  # noqa: F401
    _lib.load().mi_bn_set_small_elems(int(sys.argv[4]))
    print("bn small elems", sys.argv[4])
g = torch.Generator(device="cuda").manual_seed(7)
x = torch.randn(bs, 3, size, size, device="cuda", generator=g)
outs = {}
for nol in (False, True):
    RB.NOL = nol
    torch.manual_seed(0)
    m = get_model(name, num_classes=10).cuda()
    with torch.no_grad():
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
    acts = []
    hooks = [mod.register_forward_hook(lambda mod, i, o: acts.append(o.detach().float().clone()))
             for n_, mod in m.named_modules() if n_.count(".") == 1 and n_.startswith("layer")]
    out = m(x)
    torch.cuda.synchronize()
    outs[nol] = acts + [out.detach().float()]
    for h in hooks:
        h.remove()
print("NOL used", RB.NOL_USED[0])
for k, (a, b) in enumerate(zip(outs[False], outs[True])):
    d = (a - b).abs()
    print(k, tuple(a.shape), "max abs", float(d.max()), "rel", float(d.max() / a.abs().max()), "frac diff", float((d > 0).float().mean()))
