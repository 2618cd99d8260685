#!/usr/bin/env python3
"""Sketch encode cost vs chunk size, quantile count and segment structure (1 GPU).

Separates per-element cost (LDS bin search + LDS atomics) from per-workgroup setup and from
global-atomic contention on the per-segment totals: the same 25.5 M N(0,1) elements split as
ResNet-50's per-parameter segments, as ONE segment (every workgroup adds into the same q totals),
and as equal 64 K segments.  Prints one line per configuration: us per encode call."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from grace_amd.compressor.sketch import native_quantile_edges
from grace_amd.models.resnet import resnet50
from grace_amd.ops import _native
from grace_amd.ops.layout import SegmentLayout


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dbg = os.environ.get("GRACE_SKETCH_DBG", "0")  # honoured by builds that have the diagnostic modes
    lib = _native.lib()
    shapes = [p.shape for p in resnet50().parameters()]
    n = sum(torch.Size(s).numel() for s in shapes)
    x = torch.randn(n, device="cuda")
    layouts = {
        "resnet50": SegmentLayout.from_tensors([torch.empty(s) for s in shapes]),
        "one_segment": SegmentLayout.from_tensors([torch.empty(n)]),
        "64k_segments": SegmentLayout.from_tensors([torch.empty(65536)] * (n // 65536) + [torch.empty(n % 65536)]),
    }
    quick = os.environ.get("GRACE_SKETCH_PROBE_QUICK") == "1"  # one configuration (diagnostic sweeps)
    if quick:
        layouts = {"resnet50": layouts["resnet50"]}
    for lname, lay in layouts.items():
        for q in ((64,) if quick else (16, 64)):
            edges = native_quantile_edges(x, lay, q)
            bins = torch.empty(n, dtype=torch.uint8, device="cuda")
            means = torch.empty(lay.n_seg * q, device="cuda")
            sums = torch.zeros(lay.n_seg * q, dtype=torch.int64, device="cuda")
            cnts = torch.zeros(lay.n_seg * q, dtype=torch.int32, device="cuda")
            arrive = torch.zeros(lay.n_seg, dtype=torch.int32, device="cuda")
            for chunk in ((8192,) if quick else (2048, 8192, 32768)):
                t = lay.device_tables(x.device, chunk)
                us = timed(lambda: lib.sketch_encode(x, edges, q, bins, sums, cnts, t["seg"], t["begin"], t["end"],
                                                     arrive, t["seg_chunk_begin"], means))
                print(f"dbg={dbg:2s} {lname:13s} q={q:3d} chunk={chunk:6d} blocks={t['n_chunks']:6d}  {us:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
