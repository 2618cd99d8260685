"""FP16Compressor -- 16-bit casting (reference /root/reference/grace_dl/dist/compressor/fp16.py:6-22).

``dtype`` may be ``torch.float16`` (reference) or ``torch.bfloat16`` (same 2 bytes/element on
the wire, fp32 exponent range: no overflow when the 16-bit payload is SUM-allreduced).
Non-floating tensors pass through unchanged, as in the reference.
"""
from __future__ import annotations

import torch

from ..core import Compressor


class FP16Compressor(Compressor):
    allreduce_compatible = True

    def __init__(self, dtype: torch.dtype = torch.float16, average: bool = True):
        super().__init__(average=average)
        self.dtype = dtype

    def compress(self, tensor, name):
        dtype = tensor.dtype
        if dtype.is_floating_point:
            tensor = tensor.to(self.dtype)
        return [tensor], dtype

    def decompress(self, tensors, dtype):
        (t,) = tensors
        return t.to(dtype) if dtype.is_floating_point else t

    def decompress_reduced(self, tensors, dtype, world_size):
        (t,) = tensors
        out = t.to(dtype) if dtype.is_floating_point else t
        if self.average and world_size > 1:
            out = out.div_(world_size) if out.is_floating_point() else out // world_size
        return out

    def decompress_aggregate(self, per_rank, dtype, world_size):
        acc = per_rank[0][0].to(torch.float32 if dtype.is_floating_point else dtype)
        acc = acc.clone() if acc.data_ptr() == per_rank[0][0].data_ptr() else acc
        for p in per_rank[1:]:
            acc.add_(p[0])
        if self.average and world_size > 1:
            acc = acc.div_(world_size) if acc.is_floating_point() else acc // world_size
        return acc.to(dtype)
