"""Signum -- SignSGD with momentum (Bernstein et al., arXiv 1802.04434).

Reference: /root/reference/grace_dl/dist/compressor/signum.py:6-37 -- m = (1-beta)*x + beta*m_prev
(per-name state, first step m = x), payload sign(m) as uint8, majority-vote aggregate,
``average=False``.  Here the momentum update and the 1-bit packing are ONE kernel pass
(csrc/kernels/signbits.hip, MOM variant); the momentum buffers are checkpointable state.
"""
from __future__ import annotations

import torch

from .signsgd import SignSGDCompressor


class SignumCompressor(SignSGDCompressor):
    _state_attrs = ("steps", "momentums")

    def __init__(self, momentum: float = 0.9):
        super().__init__()
        self.momentum = momentum
        self.momentums = {}

    def _momentum(self, g, name):
        m = self.momentums.get(name)
        if m is None or m.shape != g.shape or m.device != g.device:
            m = self.momentums[name] = torch.empty_like(g)
            return m, False
        return m, True
