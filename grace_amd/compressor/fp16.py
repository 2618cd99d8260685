"""FP16Compressor -- 16-bit casting (reference /root/reference/grace_dl/dist/compressor/fp16.py:6-22).

``dtype`` may be ``torch.float16`` (reference) or ``torch.bfloat16`` (same 2 bytes/element on
the wire, fp32 exponent range: no overflow when the 16-bit payload is SUM-allreduced).
Non-floating tensors pass through unchanged, as in the reference.
"""
from __future__ import annotations

import torch

from ..core import Compressor
from ..ops import _native
from ..parallel.comm import rank_rows


class FP16Compressor(Compressor):
    allreduce_compatible = True

    def __init__(self, dtype: torch.dtype = torch.float16, average: bool = True):
        super().__init__(average=average)
        self.dtype = dtype

    def compress(self, tensor, name):
        dtype = tensor.dtype
        if dtype == torch.float32 and _native.use_native(tensor) and tensor.is_contiguous():
            out = torch.empty(tensor.shape, dtype=self.dtype, device=tensor.device)
            _native.lib().cast16(tensor.view(-1), out.view(-1), self.dtype == torch.bfloat16)
            return [out], dtype
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
        t0 = per_rank[0][0]
        if dtype == torch.float32 and _native.use_native(t0) and t0.dtype in (torch.float16, torch.bfloat16):
            base, stride, offs = rank_rows(per_rank)
            out = torch.empty(t0.shape, dtype=torch.float32, device=t0.device)
            _native.lib().decode16_sum(base[offs[0]:], stride, len(per_rank), t0.dtype == torch.bfloat16,
                                       1.0 / world_size if self.average else 1.0, out.view(-1))
            return out
        acc = per_rank[0][0].to(torch.float32 if dtype.is_floating_point else dtype)
        acc = acc.clone() if acc.data_ptr() == per_rank[0][0].data_ptr() else acc
        for p in per_rank[1:]:
            acc.add_(p[0])
        if self.average and world_size > 1:
            acc = acc.div_(world_size) if acc.is_floating_point() else acc // world_size
        return acc.to(dtype)
