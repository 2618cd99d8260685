"""ThresholdCompressor -- send every entry with |x| > threshold.

Reference: /root/reference/grace_dl/dist/compressor/threshold.py:6-27 (``torch.where`` +
gather; variable-size payload ``[values, int64 indices]``, exchanged by the size all-gather +
padding of allgather.py:15-38).  Here: one ballot-compaction kernel (csrc/kernels/sparsify.hip)
writes fp32 values + int32 flat indices into a FIXED-capacity payload with an in-band count
(grace_amd/ops/cappayload.py), with ResidualMemory fused into the same pass.  No host read of the
size anywhere, so the exchange is graph-capturable.

``capacity`` (fraction of the tensor, default 1.0 = exact reference semantics, never spills)
bounds the bytes on the wire: with capacity < 1 at most ceil(capacity * n) of the selected
entries are sent per step and the rest stay in the residual (ResidualMemory) -- which subset is
sent is unspecified on the GPU (atomic slot order).

Default threshold 0.01 (the dist helper's 256 selects nothing: survey 2.14 #19).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..core import Compressor
from ..memory.residual import ResidualMemory
from ..ops import _native
from ..ops import cappayload as P


@dataclass
class ThresholdCtx:
    numel: int
    shape: torch.Size
    dtype: torch.dtype
    cap: int


def _compact(g, thr, cap, r=None, r_valid=False, beta=1.0, gamma=1.0):
    hdr, v, i = P.sparse_payload(g.device, cap)
    if _native.use_native(g):
        mode = 1 if (r is not None and r_valid) else 0
        _native.lib().threshold_compact(g, r if mode else None, mode, beta, gamma, thr, v, i, hdr[:1], r)
        return hdr, v, i
    x = g if r is None else ((beta * r + gamma * g) if r_valid else g.clone())
    (idx,) = torch.where(x.abs() > thr)
    hdr.zero_()
    hdr[0] = idx.numel()
    hdr[1] = cap
    s = idx[:cap]
    v[: s.numel()] = x[s]
    i[: s.numel()] = s.to(torch.int32)
    if r is not None:
        r.copy_(x)
        r[s] = 0.0  # spilled entries (past the capacity) stay in the residual
    return hdr, v, i


class ThresholdCompressor(Compressor):
    def __init__(self, threshold: float = 0.01, capacity: float = 1.0):
        super().__init__(tensors_size_are_same=True)  # fixed-capacity payload
        self.threshold = threshold
        self.capacity = capacity

    def _ctx(self, tensor):
        return ThresholdCtx(tensor.numel(), tensor.shape, tensor.dtype, P.capacity(tensor.numel(), self.capacity))

    def compress(self, tensor, name):
        g = tensor.reshape(-1).float().contiguous()
        ctx = self._ctx(tensor)
        return list(_compact(g, self.threshold, ctx.cap)), ctx

    def fused_compress(self, tensor, name, memory):
        if not isinstance(memory, ResidualMemory):
            return None
        g = tensor.reshape(-1).float().contiguous()
        r, valid = memory.residual_buffer(name, g)
        ctx = self._ctx(tensor)
        return list(_compact(g, self.threshold, ctx.cap, r, valid, memory.beta, memory.gamma)), ctx

    def wire_counts(self, tensors):
        return [None, (0, [4]), (0, [4])]  # [header(selected, cap), values, indices]

    def decompress(self, tensors, ctx):
        hdr, v, i = tensors
        out = torch.zeros(ctx.numel, dtype=torch.float32, device=v.device)
        P.scatter_capped(hdr, v, i, out, 1.0, accumulate=False)
        return out.view(ctx.shape).to(ctx.dtype)

    def decompress_aggregate(self, per_rank, ctx, world_size):
        out = torch.zeros(ctx.numel, dtype=torch.float32, device=per_rank[0][1].device)
        scale = 1.0 / world_size if self.average else 1.0
        for hdr, v, i in per_rank:  # fixed rank order: identical result on every rank
            P.scatter_capped(hdr, v, i, out, scale, accumulate=True)
        return out.view(ctx.shape).to(ctx.dtype)
