"""DgcMemory -- momentum correction + local accumulation (Lin et al., DGC, arXiv 1712.01887).

Reference: /root/reference/grace_dl/dist/memory/dgc.py:7-39
  compensate: optional clip to sqrt(allreduce(sum x^2) / W); u = m*u + x; v += u; return v
  update:     u *= ~mask; v *= ~mask  (mask = elements the DgcCompressor sent)

Fixes: the reference's ``dist.all_reduce`` returns None, so clipping always raised a TypeError
(dist/memory/dgc.py:19); here the squared norms of *all* segments of a bucket are all-reduced
in ONE collective through the communicator's comm handle and clipping works.  The u/v state is
never aliased to the caller's gradient tensor (the reference aliases it on the first step).
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

    def compensate(self, tensor, name):
        if self.gradient_clipping:
            tensor = self._clip(tensor, name)
        u = self.residuals.get(name)
        if u is not None:
            u.mul_(self.momentum).add_(tensor)
        else:
            u = self.residuals[name] = tensor.clone()
        v = self.gradients.get(name)
        if v is not None:
            v.add_(u)
        else:
            v = self.gradients[name] = u.clone()
        return v

    def update(self, tensor, name, compressor, tensors_compressed, ctx):
        sel = ctx.selected  # flat indices the compressor sent
        u = self.residuals[name].view(-1)
        v = self.gradients[name].view(-1)
        u.index_fill_(0, sel, 0.0)
        v.index_fill_(0, sel, 0.0)
