"""Per-layer fp32 convolution timing for the ResNet-50 b32 step: MIOpen channels-last vs NCHW,
and 1x1 convs as plain hipBLASLt GEMMs over the channels-last activation ([N*H*W, Cin] x Wᵀ) ("mm")
and on the hand-written f32 MFMA GEMM (grace_amd.ops.conv, "mf").

Prints, for every unique conv shape (with its multiplicity in the network), fwd and fwd+bwd
ms per call for each path, and the whole-network totals weighted by multiplicity.

    python benchmarks/conv_bench.py [--batch 32] [--dtype fp32] [--iters 20]
"""
from __future__ import annotations

import argparse
import collections

import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from grace_amd.ops.conv import _Conv1x1Fn  # noqa: E402


def resnet50_convs(batch):
    """(N, Cin, H, W, Cout, k, stride) -> count, walking torchvision's ResNet-50 v1.5."""
    convs = collections.Counter()
    convs[(batch, 3, 224, 224, 64, 7, 2)] += 1
    h, cin = 56, 64
    for planes, n, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for i in range(n):
            s = stride if i == 0 else 1
            convs[(batch, cin, h, h, planes, 1, 1)] += 1
            convs[(batch, planes, h, h, planes, 3, s)] += 1
            ho = h // s
            convs[(batch, planes, ho, ho, planes * 4, 1, 1)] += 1
            if i == 0:
                convs[(batch, cin, h, h, planes * 4, 1, s)] += 1
            cin, h = planes * 4, ho
    return convs


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


class _MM1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        n, c, h, ww = x.shape
        x2 = x.permute(0, 2, 3, 1).reshape(-1, c)  # channels-last: a view
        w2 = w.view(w.shape[0], c)
        ctx.save_for_backward(x2, w2)
        ctx.shape = (n, h, ww)
        y = x2 @ w2.t()
        return y.view(n, h, ww, -1).permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gy):
        x2, w2 = ctx.saved_tensors
        n, h, ww = ctx.shape
        g2 = gy.permute(0, 2, 3, 1).reshape(-1, w2.shape[0])
        gx = (g2 @ w2).view(n, h, ww, -1).permute(0, 3, 1, 2)
        gw = (g2.t() @ x2).view(w2.shape[0], w2.shape[1], 1, 1)
        return gx, gw


PATHS = ("cl", "nchw", "mm", "mf")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False
    dt = torch.float32 if args.dtype == "fp32" else torch.bfloat16
    dev = torch.device("cuda")
    tot = collections.defaultdict(float)
    print(f"{'shape (N,Cin,H,W,Cout,k,s)':34} {'x':>2} " + " ".join(f"{p + ' ' + m:>12}" for p in PATHS
                                                            for m in ("fwd", "f+b")))
    for shp, cnt in sorted(resnet50_convs(args.batch).items(), key=lambda kv: -kv[0][4] * kv[0][1]):
        n, cin, h, w, cout, k, s = shp
        row = {}
        for path in PATHS:
            if path in ("mm", "mf") and (k != 1 or s != 1):
                continue
            mf = torch.channels_last if path != "nchw" else torch.contiguous_format
            x = torch.randn(n, cin, h, w, device=dev, dtype=dt).to(memory_format=mf).requires_grad_(True)
            wt = (torch.randn(cout, cin, k, k, device=dev, dtype=dt) * 0.05).to(memory_format=mf).requires_grad_(True)
            if path == "mm":
                f = lambda: _MM1x1.apply(x, wt)
            elif path == "mf":
                f = lambda: _Conv1x1Fn.apply(x, wt)
            else:
                f = lambda: F.conv2d(x, wt, stride=s, padding=k // 2)
            y = f()
            gy = torch.randn_like(y)
            with torch.no_grad():
                row[path + " fwd"] = timed(f, args.iters)

            def fb():
                out = f()
                gx, gw = torch.autograd.grad(out, (x, wt), gy)
            row[path + " f+b"] = timed(fb, args.iters)
            if path in ("mm", "mf"):  # numerics vs the MIOpen conv
                ref = F.conv2d(x.detach().contiguous(), wt.detach().contiguous())
                err = (y.detach() - ref).abs().max().item() / ref.abs().max().item()
                assert err < 1e-4, (shp, err)
        for key, v in row.items():
            tot[key] += cnt * v
        best_fb = min(v for kk, v in row.items() if kk.endswith("f+b"))
        tot["best f+b"] += cnt * best_fb
        tot["cl f+b (mf where 1x1 s1)"] += cnt * row.get("mf f+b", row["cl f+b"])
        print(f"{str(shp):34} {cnt:>2} " + " ".join(f"{row.get(p + ' ' + m, float('nan')):12.3f}"
                                                   for p in PATHS for m in ("fwd", "f+b")))
    print("totals (ms per network step, weighted by multiplicity):")
    for key, v in tot.items():
        print(f"  {key:30} {v:8.3f}")


if __name__ == "__main__":
    main()
