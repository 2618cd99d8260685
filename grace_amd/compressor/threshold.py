"""ThresholdCompressor -- send every entry with |x| > threshold.

Reference: /root/reference/grace_dl/dist/compressor/threshold.py:6-27 (``torch.where`` +
gather; variable-size payload ``[values, int64 indices]``, exchanged by the size all-gather +
padding of allgather.py:15-38).  Here: one ballot-compaction kernel (csrc/kernels/sparsify.hip)
writes fp32 values + int32 flat indices into a FIXED-capacity payload with an in-band count
(grace_amd/ops/cappayload.py), with ResidualMemory fused into the same pass.  No host read of the
size anywhere, so the exchange is graph-capturable.

``capacity`` (fraction of the tensor) bounds the bytes on the wire: at most ceil(capacity * n)
of the selected entries are sent per step.  ``None`` (default, "auto"):
  * with ResidualMemory fused (error feedback): 1/32 of the tensor (8n/32 + 16 bytes per rank,
    ~6 % of the uncompressed 4n), grown lagged and sync-free when a step overflows
    (ops/cappayload.py AdaptiveCapacity); entries past the capacity stay in the residual and go
    out in a later step -- spill, not loss;
  * without error feedback: 1.0 (exact reference semantics, never spills).
Which subset is sent when a step spills is unspecified on the GPU (atomic slot order).  Every
spilled payload is counted by the decode kernel in ``parallel.health.overflows()`` -- also for
steps replayed from a HIP graph, whose capacity is frozen at capture.  On the
xGMI one-shot path only each peer's selected entries move regardless (count-aware pull).

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
    name: str = ""
    adapt: bool = False


def _compact(g, thr, cap, r=None, r_valid=False, beta=1.0, gamma=1.0):
    hdr, v, i = P.sparse_payload(g.device, cap)
    if _native.use_native(g):
        from ..parallel import health as _health

        _health.init_for(g)  # spilled steps are counted by the decoder (health.overflows())
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
    AUTO_EF_RATIO = 1.0 / 32

    def __init__(self, threshold: float = 0.01, capacity=None):
        super().__init__(tensors_size_are_same=True)  # fixed-capacity payload
        self.threshold = threshold
        self.capacity = capacity
        self.adaptive = P.AdaptiveCapacity(self.AUTO_EF_RATIO) if capacity is None else None


    def _ctx(self, tensor, name, ef: bool):
        n = tensor.numel()
        if self.adaptive is not None and ef:
            cap = self.adaptive.get(name, n, n)
        else:
            cap = P.capacity(n, 1.0 if self.capacity is None else self.capacity)
        return ThresholdCtx(n, tensor.shape, tensor.dtype, cap, name, self.adaptive is not None and ef)

    def compress(self, tensor, name):
        g = tensor.reshape(-1).float().contiguous()
        ctx = self._ctx(tensor, name, ef=False)
        return list(_compact(g, self.threshold, ctx.cap)), ctx

    def fused_compress(self, tensor, name, memory):
        if not isinstance(memory, ResidualMemory):
            return None
        g = tensor.reshape(-1).float().contiguous()
        r, valid = memory.residual_buffer(name, g)
        ctx = self._ctx(tensor, name, ef=True)
        return list(_compact(g, self.threshold, ctx.cap, r, valid, memory.beta, memory.gamma)), ctx

    def _observe(self, per_rank, ctx):
        if getattr(ctx, "adapt", False):  # every rank's header: the same decision on every rank
            self.adaptive.observe(ctx.name, [p[0][:1] for p in per_rank], lambda w: w[0])

    def wire_counts(self, tensors):
        return [None, (0, [4]), (0, [4])]  # [header(selected, cap), values, indices]

    def decompress(self, tensors, ctx):
        hdr, v, i = tensors
        out = torch.zeros(ctx.numel, dtype=torch.float32, device=v.device)
        P.scatter_capped(hdr, v, i, out, 1.0, accumulate=False)
        return out.view(ctx.shape).to(ctx.dtype)

    def decompress_aggregate(self, per_rank, ctx, world_size):
        self._observe(per_rank, ctx)
        out = torch.empty(ctx.numel, dtype=torch.float32, device=per_rank[0][1].device)
        scale = 1.0 / world_size if self.average else 1.0
        # zero + the W payloads in fixed rank order: identical result on every rank
        P.decode_ranks([p[1] for p in per_rank], [p[2] for p in per_rank], [p[0] for p in per_rank], out, scale,
                       own=P.own_rank(ctx))
        return out.view(ctx.shape).to(ctx.dtype)
