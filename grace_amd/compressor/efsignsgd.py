"""EF-SignSGD (Karimireddy et al., arXiv 1901.09847).

Reference: /root/reference/grace_dl/dist/compressor/efsignsgd.py:6-33 -- payload
(mean|x|, x >= 0 as uint8), decompress mean*(2b-1), aggregate sum / lr, ``average=False``.

MI355X: per-segment mean|x| from the one-pass segment statistics kernel (which also performs
the EFSignSGDMemory compensate x = r + lr*g and stores x), then ONE sign-pack pass writes the
1-bit words and the new residual x - mean*(2b-1).  Aggregation decodes all W ranks in one pass.
Payload: [(mean, -mean) fp32 per segment | 1-bit words].
"""
from __future__ import annotations

import torch

from ..memory.residual import ResidualMemory
from ..ops import segstats as S
from ..ops import signbits as SB
from ._base import BucketCompressor


class EFSignSGDCompressor(BucketCompressor):
    reduce_by_allgather = True
    allreduce_compatible = True

    def __init__(self, lr: float):
        super().__init__(average=False)
        self.learning_rate = lr

    def _vals(self, stats, lay):
        n = lay.numels_t(stats.device).clamp_min(1)
        mean = stats[:, S.ABSSUM] / n
        return mean, -mean

    def _encode(self, g, ctx, name, memory=None):
        lay = ctx.layout
        vals, words = self.payload(g.device, [(torch.float32, (2 * lay.n_seg,)), (torch.int64, (lay.n_words,))])
        if memory is None:
            stats = S.segment_stats(g, lay)
            vt, vf = self._vals(stats, lay)
            SB.sign_pack(g, lay, words)
        else:
            r, valid = memory.residual_buffer(name, g)
            stats = S.segment_stats(g, lay, r=r, r_valid=valid, beta=memory.beta, gamma=memory.gamma, xout=r)
            vt, vf = self._vals(stats, lay)
            SB.sign_pack(r, lay, words, vT=vt, vF=vf, resid=r)
        v2 = vals.view(-1, 2)
        v2[:, 0] = vt
        v2[:, 1] = vf
        return [vals, words]

    def compress(self, tensor, name):
        ctx = self.ctx(tensor, name)
        return self._encode(self.flat(tensor), ctx, name), ctx

    def fused_compress(self, tensor, name, memory):
        if not isinstance(memory, ResidualMemory):
            return None
        ctx = self.ctx(tensor, name)
        return self._encode(self.flat(tensor), ctx, name, memory), ctx

    def aggregate_scale(self, world_size):
        return 1.0 / self.learning_rate  # reference aggregate: sum / lr

    def decompress(self, tensors, ctx):
        return self.decompress_aggregate_impl([list(tensors)], ctx, 1, 1.0)

    def decompress_aggregate_impl(self, per_rank, ctx, n_ranks, scale):
        base, stride, offs = self.rows(per_rank)
        out = self.out_buffer(ctx, base.device)
        SB.sign_unpack(base, stride, offs[1], offs[0], n_ranks, ctx.layout, out, vote=False, scale=scale)
        return self.finish(out, ctx)

    def aggregate(self, tensors):
        return super().aggregate(tensors) / self.learning_rate
