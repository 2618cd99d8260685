"""EFSignSGDMemory -- error feedback for EF-SignSGD (Karimireddy et al., 2019).

Reference: /root/reference/grace_dl/dist/memory/efsignsgd.py:4-19
  compensate: x' = residual + lr * x  (once a residual exists), update: residual = x' - dec.
It is ResidualMemory with beta = 1, gamma = lr, so it shares the fused kernels.
(The reference dist helper cannot build it -- dist/helper.py:57-74 -- grace_amd registers it.)
"""
from .residual import ResidualMemory


class EFSignSGDMemory(ResidualMemory):
    def __init__(self, lr: float):
        super().__init__(beta=1.0, gamma=lr)
        self.learning_rate = lr
