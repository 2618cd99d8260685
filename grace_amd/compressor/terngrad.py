"""TernGrad -- stochastic ternarization (Wen et al., arXiv 1705.07878).

Reference: /root/reference/grace_dl/dist/compressor/terngrad.py:8-32 -- c = 2.5*std(x),
g = clamp(x, +-c), scalar = max|g|, t = sign(g) where U[0, scalar) < |g| else 0; payload
(int8 t, scalar); decompress t*scalar.  The reference syncs the host twice (``.item()``).

MI355X (csrc/kernels/quant.hip): mean/std/max|x| of every segment from ONE statistics pass
(max|clamp(x,+-c)| = min(max|x|, c), so no second reduction), everything stays on the device,
and t travels as two 1-bit planes (nonzero, negative) = 2 bits/element instead of 8.
Payload: [bit-plane words (2 per 64 elements) | scalar fp32 per segment].
"""
from __future__ import annotations

import torch

from ..memory.residual import ResidualMemory
from ..ops import quant as Q
from ..ops import segstats as S
from ._base import BucketCompressor


class TernGradCompressor(BucketCompressor):
    reduce_by_allgather = True
    allreduce_compatible = True

    def __init__(self, clip_factor: float = 2.5):
        super().__init__()
        self.clip_factor = clip_factor

    def _encode(self, g, ctx, name, memory=None):
        lay = ctx.layout
        words, scal = self.payload(g.device, [(torch.int64, (2 * lay.n_words,)), (torch.float32, (lay.n_seg,))])
        r = None
        if memory is None:
            stats = S.segment_stats(g, lay)
            x = g
        else:
            r, valid = memory.residual_buffer(name, g)
            stats = S.segment_stats(g, lay, r=r, r_valid=valid, beta=memory.beta, gamma=memory.gamma, xout=r)
            x = r
        n = lay.numels_t(g.device).clamp_min(1)
        mean = stats[:, S.SUM] / n
        var = (stats[:, S.SUMSQ] / n - mean * mean).clamp_min(0)
        clip = self.clip_factor * torch.sqrt(var)
        torch.minimum(stats[:, S.ABSMAX], clip, out=scal)
        seed, step = self.next_rng(name, x.device)
        Q.tern_quantize(x, lay, clip, scal, seed, words, resid=r, step=step)
        return [words, scal]

    def compress(self, tensor, name):
        ctx = self.ctx(tensor, name)
        return self._encode(self.flat(tensor), ctx, name), ctx

    def fused_compress(self, tensor, name, memory):
        if not isinstance(memory, ResidualMemory):
            return None
        ctx = self.ctx(tensor, name)
        return self._encode(self.flat(tensor), ctx, name, memory), ctx

    def decompress_aggregate_impl(self, per_rank, ctx, n_ranks, scale):
        base, stride, offs = self.rows(per_rank)
        out = self.out_buffer(ctx, base.device)
        Q.tern_aggregate(base, stride, offs[0], offs[1], n_ranks, ctx.layout, out, scale)
        return self.finish(out, ctx)
