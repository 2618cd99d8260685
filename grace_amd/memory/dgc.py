"""DgcMemory -- momentum correction + local accumulation (Lin et al., DGC, arXiv 1712.01887).

Reference: /root/reference/grace_dl/dist/memory/dgc.py:7-39
  compensate: optional clip to sqrt(allreduce(sum x^2) / W); u = m*u + x; v += u; return v
  update:     u *= ~mask; v *= ~mask  (mask = elements the DgcCompressor sent)

Fixes: the reference's ``dist.all_reduce`` returns None, so clipping always raised a TypeError
(dist/memory/dgc.py:19); here the squared norms of *all* segments of a bucket are all-reduced
in ONE collective through the communicator's comm handle and clipping works.  The u/v state is
never aliased to the caller's gradient tensor (the reference aliases it on the first step).
With DgcCompressor on the GPU, compensate and update are fused into the DGC kernels
(DgcCompressor.fused_compress: one u/v pass, masking inside the compaction).
"""
from __future__ import annotations

import torch

from ..core import Memory, layout_of
from ..ops import segstats as S


class DgcMemory(Memory):
    _state_attrs = ("residuals", "gradients")

    def __init__(self, momentum: float = 0.9, gradient_clipping=False, world_size: int | None = None):
        self.momentum = momentum
        self.gradient_clipping = gradient_clipping
        self.world_size = world_size
        self.residuals = {}  # u (momentum)
        self.gradients = {}  # v (accumulated)
        self.comm = None

    def bind_comm(self, comm):
        self.comm = comm
        if self.world_size is None:
            self.world_size = comm.world_size

    def _clip(self, tensor, name):
        lay = layout_of(tensor, name)
        flat = tensor.reshape(-1).float()
        sq = S.segment_stats(flat.contiguous(), lay)[:, S.SUMSQ].contiguous()
        if self.comm is not None and self.comm.world_size > 1:
            self.comm.all_reduce(sq)
        W = self.world_size or 1
        clip = torch.sqrt(sq / W)
        c = S.expand(clip, lay).view_as(tensor)
        return torch.maximum(torch.minimum(tensor, c), -c)

    def state_buffers(self, name, g):
        """(u, v, first) flat fp32 state for the fused native path (allocated on first use)."""
        u = self.residuals.get(name)
        v = self.gradients.get(name)
        if u is None or v is None or u.numel() != g.numel() or u.device != g.device:
            u = self.residuals[name] = torch.empty_like(g, memory_format=torch.contiguous_format)
            v = self.gradients[name] = torch.empty_like(g, memory_format=torch.contiguous_format)
            return u.view(-1), v.view(-1), True
        return u.view(-1), v.view(-1), False

    def compensate(self, tensor, name):
        if self.gradient_clipping:
            tensor = self._clip(tensor, name)
        u = self.residuals.get(name)
        if u is not None:
            u.mul_(self.momentum).add_(tensor.view_as(u))
        else:
            u = self.residuals[name] = tensor.clone()
        v = self.gradients.get(name)
        if v is not None:
            v.add_(u)
        else:
            v = self.gradients[name] = u.clone()
        return v.view_as(tensor)

    def update(self, tensor, name, compressor, tensors_compressed, ctx):
        """u *= ~sent; v *= ~sent (reference dgc.py:32-39 with mask = the entries actually sent)."""
        sent = ctx.selected
        u = self.residuals[name].view(-1)
        v = self.gradients[name].view(-1)
        if isinstance(sent, tuple):  # capacity payload: (header, indices), count read on the device
            from ..ops import cappayload as P

            hdr, idx = sent
            z = self._zeros(idx.numel(), idx.device)
            P.zero_capped(hdr, idx, u, z)
            P.zero_capped(hdr, idx, v, z)
            return
        sel = sent.long()
        u.index_fill_(0, sel, 0.0)
        v.index_fill_(0, sel, 0.0)

    def _zeros(self, n, device):
        z = getattr(self, "_zbuf", None)
        if z is None or z.numel() < n or z.device != device:
            z = self._zbuf = torch.zeros(max(n, 1), dtype=torch.float32, device=device)
        return z
