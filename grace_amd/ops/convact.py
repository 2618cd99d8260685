"""``ConvBiasAct2d``: ``act(conv2d(x, w) + b)`` with the bias and ReLU as native kernels.

MIOpen returns a convolution without its bias; PyTorch then runs a broadcast add and (VGG) an
in-place ReLU, and in backward ``threshold_backward`` plus a bias-gradient reduction: four full
activation passes and three launches around every conv (``profiles/r2_workloads_fp32_kernels.txt``,
VGG-16: ≈2.7 ms of a 29 ms fp32 step).  Here the forward is one streaming pass
(``csrc/kernels/bnact.hip`` ``bias_act_fwd_kernel``) and the backward ONE pass that writes
``dz = dy * [y > 0]`` and reduces the bias gradient through the BN statistics' deterministic
arrival tree (``bias_act_bwd_kernel``).

A drop-in ``nn.Conv2d`` subclass (same parameters and state_dict keys); CPU / non-channels_last /
unsupported channel counts take the exact PyTorch path.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native


def _fusable(y: torch.Tensor) -> bool:
    if not (y.is_cuda and y.dtype in (torch.float32, torch.bfloat16) and _native.native_on(y.device)):
        return False
    c = y.shape[1]
    return (y.dim() == 4 and y.is_contiguous(memory_format=torch.channels_last) and c % 8 == 0 and c <= 2048
            and (c <= 256 or c % 256 == 0) and y.numel() > 0 and y.data_ptr() % 16 == 0)


class _BiasActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, relu):
        y = _native.lib().bias_act_fwd(x, bias.float(), bool(relu))
        ctx.relu = bool(relu)
        ctx.bias_dtype = bias.dtype
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        if dy.stride() != y.stride() or dy.data_ptr() % 16:
            dy = dy.contiguous(memory_format=torch.channels_last)
            if dy.stride() != y.stride() or dy.data_ptr() % 16:
                dy = dy.clone(memory_format=torch.channels_last)
        dz, db = _native.lib().bias_act_bwd(dy, y, ctx.relu)
        return dz, db.to(ctx.bias_dtype), None


def bias_act(x: torch.Tensor, bias: torch.Tensor, relu: bool = True) -> torch.Tensor:
    """``act(x + bias[None, :, None, None])``."""
    if _fusable(x):
        return _BiasActFn.apply(x, bias, relu)
    y = x + bias.view(1, -1, 1, 1).to(x.dtype)
    return F.relu(y) if relu else y


class ConvBiasAct2d(nn.Conv2d):
    """``nn.Conv2d`` (with bias) followed by an optional ReLU, the bias add and ReLU fused."""

    def __init__(self, *args, relu: bool = True, **kw):
        super().__init__(*args, **kw)
        if self.bias is None:
            raise ValueError("ConvBiasAct2d needs bias=True")
        self.relu = relu

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from . import conv as _conv

        if _conv.conv3x3_ok(x, self, bias_ok=True):  # implicit GEMM on the f32 MFMA kernel, autotuned vs MIOpen
            y = _conv._Conv3x3Fn.apply(x, self.weight, self.stride[0])
        else:
            y = self._conv_forward(x, self.weight, None)
        return bias_act(y, self.bias, self.relu)

    def extra_repr(self) -> str:
        return super().extra_repr() + (", relu=True" if self.relu else "")
