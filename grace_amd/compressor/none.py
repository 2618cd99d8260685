"""NoneCompressor -- no compression (reference /root/reference/grace_dl/dist/compressor/none.py)."""
from __future__ import annotations

from ..core import Compressor
from ..ops.elementwise import scale_


class NoneCompressor(Compressor):
    allreduce_compatible = True

    def compress(self, tensor, name):
        return [tensor], None

    def decompress(self, tensors, ctx):
        (tensor,) = tensors
        return tensor

    def decompress_reduced(self, tensors, ctx, world_size):
        (t,) = tensors
        if self.average and world_size > 1:
            scale_(t, 1.0 / world_size) if t.is_contiguous() else t.div_(world_size)
        return t

    def decompress_aggregate(self, per_rank, ctx, world_size):
        out = per_rank[0][0].clone()
        for p in per_rank[1:]:
            out.add_(p[0])
        if self.average and world_size > 1:
            out.div_(world_size)
        return out
