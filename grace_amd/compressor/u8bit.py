"""8-bit approximation (Dettmers, arXiv 1511.04561) -- the TF-only ``U8bitCompressor``.

Reference: /root/reference/grace_dl/tensorflow/compressor/u8bit.py:11-110 -- scale = max|x|,
bucketise |x|/scale into a fixed 128-entry table (tfp find_bins), code = bin*sign as int8;
decode table[|code|]*scale*sign.  Values outside the table range (tfp yields NaN there) are
clamped to the first/last bin here (parity unpinned for those edge values).

MI355X: the table lives in constant memory; encode is a per-element binary search
(csrc/kernels/quant.hip), max|x| per segment from the statistics pass.
Payload: [int8 codes | scale fp32 per segment].
"""
from __future__ import annotations

import torch

from ..memory.residual import ResidualMemory
from ..ops import quant as Q
from ..ops import segstats as S
from ._base import BucketCompressor


class U8bitCompressor(BucketCompressor):
    reduce_by_allgather = True
    allreduce_compatible = True

    def _encode(self, g, ctx, name, memory=None):
        lay = ctx.layout
        codes, scales = self.payload(g.device, [(torch.int8, (lay.total,)), (torch.float32, (lay.n_seg,))])
        r = None
        if memory is None:
            stats = S.segment_stats(g, lay)
            x = g
        else:
            r, valid = memory.residual_buffer(name, g)
            stats = S.segment_stats(g, lay, r=r, r_valid=valid, beta=memory.beta, gamma=memory.gamma, xout=r)
            x = r
        scales.copy_(stats[:, S.ABSMAX])
        Q.u8_encode(x, lay, scales, codes, resid=r)
        return [codes, scales]

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
        Q.u8_aggregate(base, stride, offs[0], offs[1], n_ranks, ctx.layout, out, scale)
        return self.finish(out, ctx)
