"""DGC -- Deep Gradient Compression sparsifier (Lin et al., arXiv 1712.01887).

Reference: /root/reference/grace_dl/dist/compressor/dgc.py:6-50 -- per tensor: sample 1% of
the entries uniformly, threshold = k'-th largest |sample| with k' = max(1, int(n*ratio*0.01)),
then up to 10 refinements (x1.3 if more than 1.3*ratio*n entries pass, x0.7 if fewer than
0.7*ratio*n), payload = (values, indices) of |x| >= thr; ctx carries the mask for DgcMemory.

Differences by design: the sample indices are drawn on the payload's device (the reference
indexes a GPU tensor with a CPU index tensor, survey 2.14 #11), per-segment thresholds for
flat buckets, the refinement runs on the device (csrc/kernels/dgc.hip: one count pass per
iteration, segments that converged stop counting) and the sparse payload is a FIXED-capacity
[header | fp32 values | int32 indices] buffer with the count in-band (ops/cappayload.py): no
host read of the size, so DGC steps are graph-capturable.  ``capacity`` (default 2.0 x the
summed per-segment targets) bounds the bytes on the wire; entries selected past it keep their
DgcMemory u / v and are sent later.  With DgcMemory the momentum correction, the selection and
the u / v masking run as one fused native sequence (``fused_compress``).
"""
from __future__ import annotations

import torch

from ..ops import _native
from ..ops import cappayload as P
from ..ops import dgc as D
from ._base import BucketCompressor, Ctx


class DgcCompressor(BucketCompressor):
    def __init__(self, compress_ratio: float = 0.01, sample_ratio: float = 0.01, max_iters: int = 10,
                 capacity: float = 2.0):
        super().__init__(tensors_size_are_same=True)  # fixed-capacity payload (ops/cappayload.py)
        self.compress_ratio = compress_ratio
        self.sample_ratio = sample_ratio
        self.max_iters = max_iters
        self.capacity = capacity

    def _select(self, g, ctx, name, vmask=None, umask=None, compensate=None):
        from ..parallel import health as _health

        _health.init_for(g)  # capacity overflows are counted by the decoder (health.overflows())
        cap = D.dgc_capacity(ctx.layout, self.compress_ratio, self.capacity)
        seed, step = self.next_rng(name, g.device)
        hdr, vals, idx = D.dgc_select(g, ctx.layout, self.compress_ratio, self.sample_ratio, self.max_iters,
                                      seed, cap, step, vmask, umask, compensate)
        ctx.extra["sent"] = (hdr, idx)
        return [hdr, vals, idx], ctx

    def compress(self, tensor, name):
        ctx = self.ctx(tensor, name)
        return self._select(self.flat(tensor), ctx, name)

    def fused_compress(self, tensor, name, memory):
        """DgcMemory fused: one pass u = m*u + g, v += u (csrc/kernels/dgc.hip dgc_compensate), the
        selection on v, and the u / v masking of DgcMemory.update inside the compaction."""
        from ..memory.dgc import DgcMemory

        if not isinstance(memory, DgcMemory) or not _native.use_native(tensor):
            return None
        if memory.gradient_clipping:
            tensor = memory._clip(tensor, name)
        g = self.flat(tensor)
        u, v, first = memory.state_buffers(name, g)
        ctx = self.ctx(tensor, name)
        # compensate fused into the selection: samples read v + (m u + g) on the fly and the first
        # refinement count pass writes u and v (csrc/kernels/dgc.hip) -- one pass over the bucket
        # fewer than compensate-then-select
        return self._select(g, ctx, name, vmask=v, umask=u, compensate=(memory.momentum, first))

    def wire_counts(self, tensors):
        return [None, (0, [4]), (0, [4])]  # [header(selected, cap), values, indices]

    def decompress_aggregate_impl(self, per_rank, ctx, n_ranks, scale):
        out = self.out_buffer(ctx, per_rank[0][1].device)
        # zero + the W payloads in rank order: identical on every rank
        P.decode_ranks([p[1] for p in per_rank], [p[2] for p in per_rank], [p[0] for p in per_rank], out, scale,
                       own=P.own_rank(ctx))
        return self.finish(out, ctx)


# DgcMemory (generic, unfused path) reads the sent entries from ctx.extra["sent"]
Ctx.selected = property(lambda self: self.extra["sent"])
