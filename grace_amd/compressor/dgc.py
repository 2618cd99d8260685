"""DGC -- Deep Gradient Compression sparsifier (Lin et al., arXiv 1712.01887).

Reference: /root/reference/grace_dl/dist/compressor/dgc.py:6-50 -- per tensor: sample 1% of
the entries uniformly, threshold = k'-th largest |sample| with k' = max(1, int(n*ratio*0.01)),
then up to 10 refinements (x1.3 if more than 1.3*ratio*n entries pass, x0.7 if fewer than
0.7*ratio*n), payload = (values, indices) of |x| >= thr; ctx carries the mask for DgcMemory.

Differences by design: the sample indices are drawn on the payload's device (the reference
indexes a GPU tensor with a CPU index tensor, survey 2.14 #11), per-segment thresholds for
flat buckets, the refinement runs on the device (csrc/kernels/dgc.hip: one count pass per
iteration, segments that converged stop counting) and the sparse payload is
fp32 values + int32 indices.  ``ctx.selected`` (flat indices) replaces the dense mask.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from ..core import layout_of
from ..ops import dgc as D
from ..ops import topk as K
from ._base import BucketCompressor, Ctx


class DgcCompressor(BucketCompressor):
    def __init__(self, compress_ratio: float = 0.01, sample_ratio: float = 0.01, max_iters: int = 10):
        super().__init__(tensors_size_are_same=False)
        self.compress_ratio = compress_ratio
        self.sample_ratio = sample_ratio
        self.max_iters = max_iters

    def compress(self, tensor, name):
        ctx = self.ctx(tensor, name)
        g = self.flat(tensor)
        vals, idx = D.dgc_select(g, ctx.layout, self.compress_ratio, self.sample_ratio, self.max_iters,
                                 self.next_seed(name))
        ctx.extra["selected"] = idx
        return [vals, idx], ctx

    def decompress_aggregate_impl(self, per_rank, ctx, n_ranks, scale):
        out = self.out_buffer(ctx, per_rank[0][0].device, zero=True)
        for v, i in per_rank:
            K.scatter_add(v, i, out, scale, accumulate=True)
        return self.finish(out, ctx)


# DgcMemory reads ctx.selected
Ctx.selected = property(lambda self: self.extra["selected"].long())
