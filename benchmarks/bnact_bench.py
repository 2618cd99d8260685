#!/usr/bin/env python3
"""Per-shape timing of the fused BN(+add)(+ReLU) kernels vs the stock MIOpen + elementwise path,
on every BatchNorm shape of ResNet-50 at batch 32 (bf16 or fp32, channels_last).

    python benchmarks/bnact_bench.py [--batch 32] [--iters 50] [--dtype fp32]

Columns: shape, forward / backward microseconds for the fused kernels with the opt-in
single-launch variants enabled (used where the grid fits co-resident with full blocks; V f/b =
vectors per thread, 0 = two kernels), the fused kernels on the two-kernel path (the default), and
stock (MIOpen + elementwise); the first column's effective HBM rate.
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from grace_amd.ops.bnact import BatchNormAct2d  # noqa: E402

# (C, H, W, relu, residual, count) of ResNet-50's BatchNorm layers at 224x224 input
R50 = [(64, 112, 112, True, False, 1)]
for (c, hw, n) in ((64, 56, 3), (128, 28, 4), (256, 14, 6), (512, 7, 3)):
    R50 += [(c, hw, hw, True, False, 2 * n - 1), (c, hw * (2 if c > 64 else 1), hw * (2 if c > 64 else 1), True, False, 1),
            (4 * c, hw, hw, True, True, n), (4 * c, hw, hw, False, False, 1)]


def timed(fn, iters, graph=True):
    """us per call; with graph=True, `iters` calls are captured in one HIP graph and replayed
    (no host launch overhead: the number the whole-step-graph training loop sees)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    run = fn
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        run = g.replay
        reps = 3
    else:
        reps = iters
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps if graph else iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * iters if graph else iters) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--eager", action="store_true", help="time eager launches instead of graph replays")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    a = ap.parse_args()
    dev = "cuda"
    from grace_amd.ops import _native

    lib = _native.lib()
    tot = {"ff": 0.0, "fb": 0.0, "tf": 0.0, "tb": 0.0, "uf": 0.0, "ub": 0.0}
    print(f"{'C':>5} {'H':>4} {'W':>4} relu res  cnt  V f/b | fused fwd  bwd (us) | 2-kernel fwd  bwd | "
          f"stock fwd  bwd (us) | fused GB/s fwd bwd")
    for (c, h, w, relu, res, cnt) in R50:
        m = BatchNormAct2d(c, relu=relu).to(dev)
        x = torch.randn(a.batch, c, h, w, device=dev,
                        dtype=torch.bfloat16 if a.dtype == "bf16" else torch.float32).contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x) if res else None
        dy = torch.randn_like(x)
        xg = x.clone().requires_grad_(True)
        out = {}
        res_t = {}
        for force in ("0", "2", "1"):
            os.environ["GRACE_AMD_FORCE_TORCH"] = "1" if force == "1" else "0"
            lib.bn_set_fused(force == "0")

            def fwd():
                with torch.no_grad():
                    return m(x, r)

            def fb():
                xg.grad = None
                y = m(xg, r)
                y.backward(dy)

            tf = timed(fwd, a.iters, not a.eager)
            tfb = timed(fb, a.iters, not a.eager)
            res_t[force] = (tf, tfb - tf)
        os.environ["GRACE_AMD_FORCE_TORCH"] = "0"
        lib.bn_set_fused(True)
        M = a.batch * h * w
        vf, vb = lib.bn_fused_v(M, c, False), lib.bn_fused_v(M, c, True)
        lib.bn_set_fused(False)
        nbytes = x.numel() * x.element_size()
        fwd_bytes = nbytes * (3 + (1 if res else 0))           # stats read, apply read+write (+res)
        bwd_bytes = nbytes * ((3 if relu else 2) * 2 + 1 + (1 if res else 0))  # reduce + dx reads, dx (+dres) write
        (ff, fbk), (tf2, tb2), (uf, ub) = res_t["0"], res_t["2"], res_t["1"]
        for k, v in (("ff", ff), ("fb", fbk), ("tf", tf2), ("tb", tb2), ("uf", uf), ("ub", ub)):
            tot[k] += v * cnt
        print(f"{c:5d} {h:4d} {w:4d} {str(relu)[0]:>4} {str(res)[0]:>3} {cnt:4d} {vf:2d}/{vb:<2d} | {ff:9.1f} {fbk:5.1f} | "
              f"{tf2:12.1f} {tb2:5.1f} | {uf:9.1f} {ub:5.1f} | {fwd_bytes / ff / 1e3:8.0f} {bwd_bytes / fbk / 1e3:5.0f}")
    print(f"ResNet-50 total per step (us): fused fwd {tot['ff']:.0f} bwd {tot['fb']:.0f} | two-kernel fwd {tot['tf']:.0f} "
          f"bwd {tot['tb']:.0f} | stock fwd {tot['uf']:.0f} bwd {tot['ub']:.0f}")
    print(f"single-launch spin timeouts: {lib.bn_spin_timeouts()}")


if __name__ == "__main__":
    main()
