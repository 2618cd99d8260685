"""Microbench: W-rank sparse decode of a ResNet-50-sized bucket (n = 25.56 M, Top-K 1 %):
one-launch rank-ordered decode (csrc/kernels/sparse_decode.hip) vs the zero fill + W scatter
launches it replaced.  Per-call GPU time from HIP events over 50 back-to-back calls, eager and
replayed from a HIP graph (the bench's whole-step graph issues it as one node)."""
import torch

from grace_amd.ops import _native
from grace_amd.ops import cappayload as P

n, k = 25_557_032, 255_570
lib = _native.lib()
out = torch.empty(n, device="cuda")


def old(vals, idxs, scale):
    out.zero_()
    for v, i in zip(vals, idxs):
        lib.sparse_scatter_add(v, i, out, scale, True)


def new(vals, idxs, scale):
    P.decode_ranks(vals, idxs, [None] * len(vals), out, scale)


def timed(fn, *a, reps=50):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn(*a)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn(*a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        fn(*a)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn(*a)
    e1.record()
    torch.cuda.synchronize()
    eager = e0.elapsed_time(e1) / reps * 1000
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return eager, e0.elapsed_time(e1) / reps * 1000


print(f"n = {n}, k = {k} per rank; us per decode (eager / graph-replayed)")
for W in (1, 2, 4, 8):
    gen = torch.Generator(device="cuda").manual_seed(W)
    vals = [torch.randn(k, device="cuda", generator=gen) for _ in range(W)]
    idxs = [torch.randperm(n, device="cuda", generator=gen)[:k].to(torch.int32) for _ in range(W)]
    new(vals, idxs, 1.0 / W)
    a = out.clone()
    old(vals, idxs, 1.0 / W)
    same = torch.equal(a, out)
    to = timed(old, vals, idxs, 1.0 / W)
    tn = timed(new, vals, idxs, 1.0 / W)
    print(f"W={W}: zero + {W} scatters {to[0]:8.1f} / {to[1]:8.1f}   one launch {tn[0]:8.1f} / {tn[1]:8.1f}"
          f"   bit-identical {same}", flush=True)
