"""ResidualMemory -- classic error feedback.

Reference: /root/reference/grace_dl/dist/memory/residual.py:4-20
  compensate: x' = beta * residual[name] + gamma * x   (only once a residual exists)
  update:     residual[name] = x' - decompress(compress(x'))

On MI355X the common pairs (Top-K, Random-K, sign/1-bit families, QSGD, ...) never take the
generic path below: the compressor's ``fused_compress`` computes x', the payload and the new
residual in its own kernel pass (one read of g and r, one write of r).  The generic path is
kept for user compressors and for the CPU oracle.
"""
from __future__ import annotations

from ..core import Memory
from ..ops.elementwise import axpby


class ResidualMemory(Memory):
    _state_attrs = ("residuals",)

    def __init__(self, beta: float = 1.0, gamma: float = 1.0):
        self.residuals = {}
        self.beta = beta
        self.gamma = gamma

    def compensate(self, tensor, name):
        r = self.residuals.get(name)
        if r is not None:
            return axpby(r, tensor, self.beta, self.gamma)
        return tensor

    def update(self, tensor, name, compressor, tensors_compressed, ctx):
        dec = compressor.decompress(tensors_compressed, ctx)
        self.residuals[name] = tensor - dec

    # hooks used by fused compressors -------------------------------------------------
    def residual_buffer(self, name, like):
        """(buffer, valid) -- the persistent residual buffer for ``name`` (allocated on first
        use; ``valid`` is False until a residual was stored)."""
        r = self.residuals.get(name)
        if r is None or r.shape != like.shape or r.device != like.device:
            import torch

            r = torch.empty_like(like, memory_format=torch.contiguous_format)
            self.residuals[name] = r
            return r, False
        return r, True
