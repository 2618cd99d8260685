"""ThresholdCompressor -- send every entry with |x| > threshold.

Reference: /root/reference/grace_dl/dist/compressor/threshold.py:6-27 (``torch.where`` +
gather; variable-size payload ``[values, int64 indices]``).  Here: one ballot-compaction kernel
(csrc/kernels/sparsify.hip) producing fp32 values + int32 flat indices into a capacity buffer,
with ResidualMemory fused into the same pass.  The element count is read back once (the
payload size is data dependent; the reference pays the same sync inside ``torch.where``).

Default threshold 0.01 (the dist helper's 256 selects nothing: survey 2.14 #19).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..core import Compressor
from ..memory.residual import ResidualMemory
from ..ops import _native
from ..ops import topk as K
from ..parallel.comm import PayloadBuilder


@dataclass
class ThresholdCtx:
    numel: int
    shape: torch.Size
    dtype: torch.dtype


def _compact(g, thr, r=None, r_valid=False, beta=1.0, gamma=1.0):
    n = g.numel()
    if _native.use_native(g):
        cap_v = torch.empty(n, dtype=torch.float32, device=g.device)
        cap_i = torch.empty(n, dtype=torch.int32, device=g.device)
        cnt = torch.zeros(1, dtype=torch.int32, device=g.device)
        mode = 1 if (r is not None and r_valid) else 0
        _native.lib().threshold_compact(g, r if mode else None, mode, beta, gamma, thr, cap_v, cap_i, cnt, r)
        s = int(cnt.item())
        pb = PayloadBuilder(g.device, [(torch.float32, (s,)), (torch.int32, (s,))])
        v, i = pb.tensors
        # order inside the payload is arbitrary (wave atomics); decompress is order-independent
        if s:
            v.copy_(cap_v[:s])
            i.copy_(cap_i[:s])
        return v, i
    x = g if r is None else ((beta * r + gamma * g) if r_valid else g.clone())
    (idx,) = torch.where(x.abs() > thr)
    pb = PayloadBuilder(g.device, [(torch.float32, (idx.numel(),)), (torch.int32, (idx.numel(),))])
    v, i = pb.tensors
    v.copy_(x[idx])
    i.copy_(idx)
    if r is not None:
        r.copy_(x)
        r[idx] = 0.0
    return v, i


class ThresholdCompressor(Compressor):
    def __init__(self, threshold: float = 0.01):
        super().__init__(tensors_size_are_same=False)
        self.threshold = threshold

    def compress(self, tensor, name):
        g = tensor.reshape(-1).float().contiguous()
        v, i = _compact(g, self.threshold)
        return [v, i], ThresholdCtx(tensor.numel(), tensor.shape, tensor.dtype)

    def fused_compress(self, tensor, name, memory):
        if not isinstance(memory, ResidualMemory):
            return None
        g = tensor.reshape(-1).float().contiguous()
        r, valid = memory.residual_buffer(name, g)
        v, i = _compact(g, self.threshold, r, valid, memory.beta, memory.gamma)
        return [v, i], ThresholdCtx(tensor.numel(), tensor.shape, tensor.dtype)

    def decompress(self, tensors, ctx):
        v, i = tensors
        out = torch.zeros(ctx.numel, dtype=torch.float32, device=v.device)
        K.scatter_add(v, i, out, 1.0, accumulate=False)
        return out.view(ctx.shape).to(ctx.dtype)

    def decompress_aggregate(self, per_rank, ctx, world_size):
        out = torch.zeros(ctx.numel, dtype=torch.float32, device=per_rank[0][0].device)
        scale = 1.0 / world_size if self.average else 1.0
        for v, i in per_rank:
            K.scatter_add(v, i, out, scale, accumulate=True)
        return out.view(ctx.shape).to(ctx.dtype)
