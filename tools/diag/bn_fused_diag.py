#!/usr/bin/env python3
"""Single-launch vs two-kernel BN paths on one shape: per-output differences and, for d(residual),
the fp32 pre-activation at the mismatching elements (ReLU-boundary flips vs real errors).

    python tools/diag/bn_fused_diag.py [N C H W]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from grace_amd.ops import _native  # noqa: E402
from grace_amd.ops.bnact import BatchNormAct2d  # noqa: E402


def run(fused, x, res, dy, c):
    lib = _native.lib()
    lib.bn_set_fused(fused)
    torch.manual_seed(0)
    m = BatchNormAct2d(c, relu=True).cuda()
    with torch.no_grad():
        m.weight.copy_(torch.linspace(0.5, 1.5, c))
        m.bias.copy_(torch.linspace(-0.1, 0.1, c))
    xx = x.clone().requires_grad_(True)
    rr = res.clone().requires_grad_(True)
    y = m(xx, rr)
    y.backward(dy)
    torch.cuda.synchronize()
    lib.bn_set_fused(True)
    return dict(y=y.detach(), dx=xx.grad, dres=rr.grad, dw=m.weight.grad, db=m.bias.grad, rm=m.running_mean,
                rv=m.running_var)


def main():
    n, c, h, w = (int(v) for v in sys.argv[1:5]) if len(sys.argv) >= 5 else (32, 128, 28, 28)
    g = torch.Generator().manual_seed(0)
    cl = torch.channels_last
    x = (torch.randn(n, c, h, w, generator=g) * 2 + 0.5).cuda().bfloat16().contiguous(memory_format=cl)
    res = torch.randn(n, c, h, w, generator=g).cuda().bfloat16().contiguous(memory_format=cl)
    dy = torch.randn(n, c, h, w, generator=g).cuda().bfloat16().contiguous(memory_format=cl)
    M = n * h * w
    lib = _native.lib()
    print("V fwd/bwd:", lib.bn_fused_v(M, c, False), lib.bn_fused_v(M, c, True))
    a, b = run(True, x, res, dy, c), run(False, x, res, dy, c)
    for k in a:
        d = (a[k].float() - b[k].float()).abs()
        print(f"{k:5s} max|single-two| {d.max().item():.3e}  n_diff {(d > 0).sum().item()}")
    # fp32 reference pre-activation
    xf = x.float()
    mean = xf.mean(dim=(0, 2, 3), keepdim=True)
    var = xf.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
    wt = torch.linspace(0.5, 1.5, c, device="cuda").view(1, c, 1, 1)
    bs = torch.linspace(-0.1, 0.1, c, device="cuda").view(1, c, 1, 1)
    z0 = (xf - mean) / torch.sqrt(var + 1e-5) * wt + bs + res.float()
    dres0 = dy.float() * (z0 > 0)
    for name, r in (("single", a), ("two", b)):
        bad = (r["dres"].float() - dres0).abs() > 1e-2
        idx = bad.nonzero()[:8].tolist()
        print(f"{name}: dres mismatches {int(bad.sum())}; first at {idx}")
        for i in idx[:4]:
            print("   z0", z0[tuple(i)].item(), "y", r["y"][tuple(i)].item(), "dres", r["dres"][tuple(i)].item(),
                  "dy", dy[tuple(i)].item())
    print("spin timeouts", lib.bn_spin_timeouts())


if __name__ == "__main__":
    main()
