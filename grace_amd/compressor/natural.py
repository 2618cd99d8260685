"""Natural compression (Horvath et al., arXiv 1905.10988).

Reference: /root/reference/grace_dl/dist/compressor/natural.py:9-40 (CuPy + DLPack):
round the fp32 exponent up with probability mantissa/2^23, clip the biased exponent to
[18, 145], send sign | (exponent - 18) as one byte; decode +-2^(e+18-127), 0 for code e < 1.

MI355X: one Philox elementwise pass (csrc/kernels/quant.hip) -- no CuPy, no DLPack round trip,
residual fused when paired with ResidualMemory; all W ranks decoded + summed in one pass.
"""
from __future__ import annotations

import torch

from ..memory.residual import ResidualMemory
from ..ops import quant as Q
from ..ops.elementwise import axpby
from ._base import BucketCompressor


class NaturalCompressor(BucketCompressor):
    reduce_by_allgather = True
    allreduce_compatible = True

    def _encode(self, g, ctx, name, memory=None):
        (codes,) = self.payload(g.device, [(torch.uint8, (ctx.layout.total,))])
        if memory is None:
            seed, step = self.next_rng(name, g.device)
            Q.natural_encode(g, seed, codes, step=step)
        else:
            r, valid = memory.residual_buffer(name, g)
            if valid:
                axpby(r, g, memory.beta, memory.gamma, out=r)
            else:
                r.copy_(g)
            seed, step = self.next_rng(name, r.device)
            Q.natural_encode(r, seed, codes, resid=r, step=step)
        return [codes]

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
        Q.natural_aggregate(base[offs[0]:], stride, n_ranks, out, scale)
        return self.finish(out, ctx)
