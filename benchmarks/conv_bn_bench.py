#!/usr/bin/env python3
"""Conv1x1 -> BatchNorm forward pieces, timed one at a time on the ResNet-50 b32 1x1 shapes:
the MFMA GEMM with and without the BN-statistics epilogue (per tile shape), the BN forward from
a statistics pass (bn_act_fwd) and from the GEMM partials (bn_act_fwd_partials = fold + apply).
Shows what the fused conv_bn_act path (grace_amd/ops/conv.py) saves or costs per piece.

    python benchmarks/conv_bn_bench.py [--iters 20]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grace_amd.ops import _native  # noqa: E402
from benchmarks.gemm_bench import SHAPES, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    C = _native.lib()
    print(f"{'shape (N,Cin,H,W,Cout)':28s} tile {'gemm':>7s} {'+stats':>7s} {'bn_fwd':>7s} {'bn_part':>7s}  (ms)")
    for (nb, cin, h, w, cout) in SHAPES:
        m = nb * h * w
        x = torch.randn(m, cin, device=dev)
        wt = torch.randn(cout, cin, device=dev) / cin ** 0.5
        y = torch.empty(m, cout, device=dev)
        part = torch.empty(((m + 63) // 64) * 2 * cout, device=dev)
        g, b = torch.ones(cout, device=dev), torch.zeros(cout, device=dev)
        rm, rv = torch.zeros(cout, device=dev), torch.ones(cout, device=dev)
        nbt = torch.zeros((), dtype=torch.int64, device=dev)
        t_bn = timed(lambda: C.bn_act_fwd(y, None, g, b, rm, rv, nbt, 0.1, 1e-5, True), a.iters)
        for tile in (1, 2, 3, 4):
            t_g = timed(lambda: C.gemm_f32(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 1, tile, None), a.iters)
            t_s = timed(lambda: C.gemm_f32(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 1, tile, part), a.iters)
            tiles = C.gemm_f32(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 1, tile, part)
            t_p = timed(lambda: C.bn_act_fwd_partials(y, None, part, tiles, g, b, rm, rv, nbt, 0.1, 1e-5, True),
                        a.iters)
            print(f"{str((nb, cin, h, w, cout)):28s} t{tile}   {t_g:7.3f} {t_s:7.3f} {t_bn:7.3f} {t_p:7.3f}")
        # parity of the statistics: fold of the partials vs the statistics pass
        tiles = C.gemm_f32(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 1, 4, part)
        y1, s1, _ = C.bn_act_fwd(y, None, g, b, rm, rv, nbt, 0.1, 1e-5, True)[:3]
        y2, s2, _ = C.bn_act_fwd_partials(y, None, part, tiles, g, b, rm, rv, nbt, 0.1, 1e-5, True)
        err = float((s1[:2 * cout] - s2[:2 * cout]).abs().max() / s1[:2 * cout].abs().max().clamp_min(1e-30))
        print(f"{'':28s} stats rel err (mean|invstd) {err:.2e}")


if __name__ == "__main__":
    main()
