"""PowerSGDMemory -- error feedback for PowerSGD (Vogels et al., NeurIPS 2019).

Reference: /root/reference/grace_dl/dist/memory/powersgd.py:6-37
  compensate: 1-D tensors pass; else x += residual (IN PLACE into p.grad) once seen, and a
              fresh N(0,1) Q (m x r) is drawn into the shared ``q_memory`` every step
  update:     residual = x - P Q^T

Here: compensation is out-of-place (the reference mutates the caller's gradient, survey 2.14
#6); Q is owned by the compressor (``PowerSGDCompressor.q_memory``), the memory only asks it
to redraw unless ``warm_start`` (the paper's reuse of the previous Q) is enabled.  For flat
buckets the residual is kept for the whole bucket; 1-D segments have zero residual.
"""
from __future__ import annotations

from ..core import Memory
from ..ops.elementwise import axpby


class PowerSGDMemory(Memory):
    _state_attrs = ("residuals",)

    def __init__(self, q_memory=None, compress_rank: int = 1, warm_start: bool = False):
        self.q_memory = q_memory if q_memory is not None else {}
        self.compress_rank = compress_rank
        self.warm_start = warm_start
        self.residuals = {}

    def compensate(self, tensor, name):
        if tensor.dim() == 1 and name not in self.residuals:
            # reference: 1-D tensors are never compensated (unless they are a flat bucket)
            from ..core import _LAYOUTS

            if name not in _LAYOUTS:
                return tensor
        if not self.warm_start:
            self.q_memory.pop(name, None)  # compressor draws a fresh Q
        r = self.residuals.get(name)
        if r is not None:
            return axpby(r, tensor, 1.0, 1.0)
        return tensor

    def update(self, tensor, name, compressor, tensors_compressed, ctx):
        if ctx is None:
            return
        self.residuals[name] = tensor - compressor.decompress(tensors_compressed, ctx)
