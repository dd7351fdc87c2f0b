#!/usr/bin/env python
"""GPU determinism probes of the native training path (no engine):

  A  the same forward repeated on unchanged parameters -> identical losses?
  B  two copies of one model trained in lockstep (fwd/bwd of each, then both optimizer steps)
     with stock SGD -> identical losses / gradients per step?
  C  the same two copies trained one after the other -> identical trajectories?

    python tools/determinism_check.py [--model resnet18] [--batch 32] [--size 32] [--steps 4]
"""
import argparse
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    from mi355x_dp.models import get_model
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m0 = get_model(a.model, num_classes=10).to(dev)
    crit = torch.nn.CrossEntropyLoss()
    g = torch.Generator(device=dev).manual_seed(1)
    data = [(torch.randn(a.batch, 3, a.size, a.size, device=dev, generator=g),
             torch.randint(0, 10, (a.batch,), device=dev, generator=g)) for _ in range(a.steps)]

    m = copy.deepcopy(m0)
    la = [float(crit(m(data[0][0]), data[0][1]).detach()) for _ in range(5)]
    print("A repeated forward losses:", la, flush=True)

    def run_lockstep():
        m1, m2 = copy.deepcopy(m0), copy.deepcopy(m0)
        o1 = torch.optim.SGD(m1.parameters(), lr=0.01, momentum=0.9)
        o2 = torch.optim.SGD(m2.parameters(), lr=0.01, momentum=0.9)
        out = []
        for s, (x, y) in enumerate(data):
            ls = []
            for mm, oo in ((m1, o1), (m2, o2)):
                oo.zero_grad()
                loss = crit(mm(x), y)
                loss.backward()
                ls.append(float(loss.detach()))
            gd = max(((rel(p1.grad, p2.grad), n) for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters())))
            o1.step()
            o2.step()
            out.append(ls)
            print(f"B step {s}: losses {ls[0]:.6f} {ls[1]:.6f} worst grad diff {gd[0]:.3g} {gd[1]}", flush=True)
        return out

    def csum(ts):
        return [float(t.detach().double().abs().sum()) for t in ts]

    def run_single(tag):
        mm = copy.deepcopy(m0)
        oo = torch.optim.SGD(mm.parameters(), lr=0.01, momentum=0.9)
        ls, trace = [], []
        for s, (x, y) in enumerate(data):
            oo.zero_grad()
            p_before = csum(mm.parameters())
            with torch.no_grad():
                l_nograd = float(crit(mm(x), y))
            loss = crit(mm(x), y)
            l_again = float(crit(mm(x), y).detach())
            loss.backward()
            g = csum(p.grad for p in mm.parameters())
            oo.step()
            ls.append(float(loss.detach()))
            trace.append((p_before, g))
            print(f"C{tag} step {s}: loss {ls[-1]:.6f} (no-grad fwd {l_nograd:.6f}, 2nd fwd {l_again:.6f}) "
                  f"param sum {sum(p_before):.9g} grad sum {sum(g):.9g}", flush=True)
        return ls, trace

    b = run_lockstep()
    (c1, t1), (c2, t2) = run_single(1), run_single(2)
    names = [n for n, _ in m0.named_parameters()]
    for s, ((p1, g1), (p2, g2)) in enumerate(zip(t1, t2)):
        dp = [n for n, u, v in zip(names, p1, p2) if u != v]
        dg = [n for n, u, v in zip(names, g1, g2) if u != v]
        print(f"C step {s}: params differing before the step {dp[:5]} ({len(dp)}); grads differing {dg[:5]} "
              f"({len(dg)})", flush=True)
    print("C sequential trajectories:", [round(v, 6) for v in c1], [round(v, 6) for v in c2], flush=True)

    # D: sensitivity of the training trajectory to a 1e-7 relative perturbation of the stem weight
    # -- the native model, and a stock-torch fp32 ResNet-18 of the same architecture (MIOpen convs)
    def stock_resnet18():
        import torch.nn as nn

        class Basic(nn.Module):
            def __init__(self, cin, cout, stride):
                super().__init__()
                self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
                self.bn1 = nn.BatchNorm2d(cout)
                self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
                self.bn2 = nn.BatchNorm2d(cout)
                self.down = None
                if stride != 1 or cin != cout:
                    self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

            def forward(self, x):
                o = torch.relu(self.bn1(self.conv1(x)))
                o = self.bn2(self.conv2(o))
                return torch.relu(o + (x if self.down is None else self.down(x)))

        layers = [nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(3, 2, 1)]
        cin = 64
        for cout, s in ((64, 1), (128, 2), (256, 2), (512, 2)):
            layers += [Basic(cin, cout, s), Basic(cout, cout, 1)]
            cin = cout
        layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(512, 10)]
        return nn.Sequential(*layers)

    def trajectory(mm, perturb):
        mm = copy.deepcopy(mm)
        if perturb:
            with torch.no_grad():
                w = next(mm.parameters())
                w.mul_(1 + 1e-7 * torch.randn(w.shape, device=w.device, generator=torch.Generator(device=w.device).manual_seed(5)))
        oo = torch.optim.SGD(mm.parameters(), lr=0.01, momentum=0.9)
        ls = []
        for x, y in data:
            oo.zero_grad()
            loss = crit(mm(x), y)
            loss.backward()
            oo.step()
            ls.append(round(float(loss.detach()), 6))
        return ls

    torch.manual_seed(0)
    st = stock_resnet18().to(dev)
    print("D native: base", trajectory(m0, False), "perturbed", trajectory(m0, True), flush=True)
    print("D stock fp32: base", trajectory(st, False), "perturbed", trajectory(st, True), flush=True)
    ok = len(set(la)) == 1 and all(abs(x - y) < 1e-3 for x, y in b) and \
        all(abs(x - y) < 1e-3 for x, y in zip(c1, c2))
    print("DETERMINISM_CHECK", "ok" if ok else "FAIL")


if __name__ == "__main__":
    main()
