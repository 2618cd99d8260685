"""Per-direction fp32 timing of ResNet-50's stride-1 1x1 convolutions: MIOpen (channels_last,
find on) vs the hand-written f32 MFMA GEMM (csrc/kernels/gemm_f32.hip), for the forward, the
data gradient and the weight gradient separately -- to pick the faster engine per direction.

    python benchmarks/conv_dir_bench.py [--iters 30]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.conv_bench import resnet50_convs, timed  # noqa: E402
from grace_amd.ops.conv import _splits, gemm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    conv_bwd = torch.ops.aten.convolution_backward
    tot = {k: 0.0 for k in ("mi_f", "mi_d", "mi_w", "mf_f", "mf_d", "mf_w", "best")}
    print(f"{'shape (N,Cin,H,W,Cout)':28} {'x':>2} {'MIO fwd':>8} {'MIO dx':>8} {'MIO dw':>8} "
          f"{'MF fwd':>8} {'MF dx':>8} {'MF dw':>8}")
    for (n, cin, h, w, cout, k, s), cnt in sorted(resnet50_convs(a.batch).items(), key=lambda kv: -kv[0][4] * kv[0][1]):
        if k != 1 or s != 1:
            continue
        m = n * h * w
        x = torch.randn(n, cin, h, w, device=dev).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, 1, 1, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, cout, h, w, device=dev).contiguous(memory_format=torch.channels_last)
        w2 = wt.reshape(cout, cin).contiguous()
        y = torch.empty_like(dy)
        dx = torch.empty_like(x)
        dw = torch.empty(cout, cin, device=dev)
        args = (None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1)
        t = {
            "mi_f": timed(lambda: torch.nn.functional.conv2d(x, wt), a.iters),
            "mi_d": timed(lambda: conv_bwd(dy, x, wt, *args, [True, False, False]), a.iters),
            "mi_w": timed(lambda: conv_bwd(dy, x, wt, *args, [False, True, False]), a.iters),
            "mf_f": timed(lambda: gemm(x, True, cin, w2, True, cin, y, cout, m, cout, cin, 0), a.iters),
            "mf_d": timed(lambda: gemm(dy, True, cout, w2, False, cin, dx, cin, m, cin, cout, 0), a.iters),
            "mf_w": timed(lambda: gemm(dy, False, cout, x, False, cin, dw, cin, cout, cin, m, _splits(cout, cin, m)),
                          a.iters),
        }
        for kk, v in t.items():
            tot[kk] += cnt * v
        tot["best"] += cnt * (min(t["mi_f"], t["mf_f"]) + min(t["mi_d"], t["mf_d"]) + min(t["mi_w"], t["mf_w"]))
        print(f"{str((n, cin, h, w, cout)):28} {cnt:>2} " + " ".join(f"{t[kk]:8.3f}" for kk in
                                                                  ("mi_f", "mi_d", "mi_w", "mf_f", "mf_d", "mf_w")))
    print("totals per step (ms): " + ", ".join(f"{k} {v:.3f}" for k, v in tot.items()))
    print(f"MIOpen all {tot['mi_f'] + tot['mi_d'] + tot['mi_w']:.3f}  MFMA all {tot['mf_f'] + tot['mf_d'] + tot['mf_w']:.3f}  "
          f"best-of per direction {tot['best']:.3f}")


if __name__ == "__main__":
    main()
