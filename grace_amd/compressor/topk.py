"""TopKCompressor -- keep the k = max(1, int(n * ratio)) largest-magnitude entries per tensor.

Reference: /root/reference/grace_dl/dist/compressor/topk.py:6-36 (torch.topk(|x|, k) + gather;
decompress = scatter into zeros).  Wire format: ONE int32 buffer of 2K words
[fp32 values | int32 flat indices] (8 B/element instead of 12, the TF layout
tensorflow/compressor/topk.py:32-35).

MI355X kernels (csrc/kernels/topk.hip):
* compress: segmented exact radix select (3 LDS-histogram passes + per-segment digit select)
  and a wave-ballot compaction -- all parameters of a bucket in ~7 launches.
* ``fused_compress`` with ResidualMemory / EFSignSGDMemory: the compensate
  x = beta*r + gamma*g happens in the first histogram pass and the new residual (x with the
  sent entries zeroed) is written by the compaction pass: the reference's second decompress
  (residual.py:17) disappears.
* ``decompress_aggregate``: the W payloads added in fixed rank order into the zeroed bucket
  (ops/cappayload.py decode_ranks: fill + atomic-free scatters), with the 1/W average folded in
  -> bitwise identical on every rank.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import torch

from ..core import Compressor, layout_of
from ..memory.residual import ResidualMemory
from ..ops import cappayload as P
from ..ops import topk as K
from ..ops.layout import SegmentLayout


@dataclass
class TopKCtx:
    layout: SegmentLayout
    ks: Tuple[int, ...]
    numel: int
    shape: torch.Size
    device: torch.device
    dtype: torch.dtype
    out: object = None  # optional destination (see compressor._base.Ctx.out)


class TopKCompressor(Compressor):
    def __init__(self, compress_ratio: float):
        super().__init__()
        if not 0.0 < compress_ratio <= 1.0:
            raise ValueError("compress_ratio must be in (0, 1]")
        self.compress_ratio = compress_ratio

    def _prep(self, tensor, name):
        lay = layout_of(tensor, name)
        ks = K.k_per_segment(lay, self.compress_ratio)
        ctx = TopKCtx(lay, ks, tensor.numel(), tensor.shape, tensor.device, tensor.dtype)
        g = tensor.reshape(-1)
        if g.dtype != torch.float32:
            g = g.float()
        return g.contiguous(), ctx

    def compress(self, tensor, name):
        g, ctx = self._prep(tensor, name)
        vals, idx = K.topk_ef(g, ctx.layout, ctx.ks, key=name)
        return [vals, idx], ctx

    def fused_compress(self, tensor, name, memory):
        if not isinstance(memory, ResidualMemory):
            return None
        g, ctx = self._prep(tensor, name)
        r, valid = memory.residual_buffer(name, g)
        vals, idx = K.topk_ef(g, ctx.layout, ctx.ks, resid=r, resid_valid=valid, beta=memory.beta,
                              gamma=memory.gamma, key=name)
        return [vals, idx], ctx

    def decompress(self, tensors, ctx):
        vals, idx = tensors
        out = torch.zeros(ctx.numel, dtype=torch.float32, device=vals.device)
        K.scatter_add(vals, idx, out, 1.0, accumulate=False)
        return out.view(ctx.shape).to(ctx.dtype)

    def decompress_aggregate(self, per_rank, ctx, world_size):
        from ._base import BucketCompressor

        out = BucketCompressor.out_buffer(ctx, per_rank[0][0].device) if ctx.dtype == torch.float32 \
            else torch.empty(ctx.numel, dtype=torch.float32, device=per_rank[0][0].device)
        scale = (1.0 / world_size) if self.average else 1.0
        # zero + every rank's scatter in fixed rank order -> identical on every rank
        P.decode_ranks([p[0] for p in per_rank], [p[1] for p in per_rank], [None] * len(per_rank), out, scale)
        return out.view(ctx.shape).to(ctx.dtype)

