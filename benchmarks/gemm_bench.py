#!/usr/bin/env python3
"""fp32 GEMM throughput: the hand-written MFMA GEMM (csrc/kernels/gemm_f32.hip) vs hipBLASLt
(torch.mm) on the ResNet-50 1x1-conv GEMM shapes (channels_last [M = N*H*W, C] views) and a square
reference shape.  Prints ms and TFLOP/s per direction (fwd: M x Cout x Cin; dgrad: M x Cin x Cout;
wgrad: Cout x Cin x M).

    python benchmarks/gemm_bench.py [--iters 20] [--shapes all|square]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grace_amd.ops.conv import _splits, gemm  # noqa: E402

# (N, Cin, H, W, Cout) of the stride-1 1x1 convs of ResNet-50 at batch 32
SHAPES = [(32, 64, 56, 56, 256), (32, 256, 56, 56, 64), (32, 64, 56, 56, 64), (32, 128, 28, 28, 512),
          (32, 512, 28, 28, 128), (32, 256, 14, 14, 1024), (32, 1024, 14, 14, 256), (32, 512, 7, 7, 2048),
          (32, 2048, 7, 7, 512)]


def timed(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="all")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cuda.matmul.allow_tf32 = False
    print(f"{'shape (N,Cin,H,W,Cout)':28s} {'dir':5s} {'mfma ms':>8s} {'TF/s':>6s} {'blaslt ms':>9s} {'TF/s':>6s}")
    if a.shapes in ("all", "square"):
        n = 4096
        A = torch.randn(n, n, device=dev)
        B = torch.randn(n, n, device=dev)
        C = torch.empty(n, n, device=dev)
        t1 = timed(lambda: gemm(A, True, n, B, True, n, C, n, n, n, n, 1), a.iters)
        t2 = timed(lambda: torch.mm(A, B.t()), a.iters)
        f = 2 * n ** 3 / 1e9
        print(f"{'square 4096^3':28s} {'-':5s} {t1:8.3f} {f / t1:6.1f} {t2:9.3f} {f / t2:6.1f}")
    if a.shapes == "square":
        return
    for (nb, cin, h, w, cout) in SHAPES:
        m = nb * h * w
        x = torch.randn(m, cin, device=dev)
        wt = torch.randn(cout, cin, device=dev)
        dy = torch.randn(m, cout, device=dev)
        y = torch.empty(m, cout, device=dev)
        dx = torch.empty(m, cin, device=dev)
        dw = torch.empty(cout, cin, device=dev)
        f = 2 * m * cin * cout / 1e9
        rows = [
            ("fwd", lambda: gemm(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 0), lambda: torch.mm(x, wt.t())),
            ("dgrad", lambda: gemm(dy, True, cout, wt, False, cin, dx, cin, m, cin, cout, 0), lambda: torch.mm(dy, wt)),
            ("wgrad", lambda: gemm(dy, False, cout, x, False, cin, dw, cin, cout, cin, m, _splits(cout, cin, m)),
             lambda: torch.mm(dy.t(), x)),
        ]
        for d, f1, f2 in rows:
            t1, t2 = timed(f1, a.iters), timed(f2, a.iters)
            print(f"{str((nb, cin, h, w, cout)):28s} {d:5s} {t1:8.3f} {f / t1:6.1f} {t2:9.3f} {f / t2:6.1f}")


if __name__ == "__main__":
    main()
