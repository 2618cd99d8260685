"""``MaxPool2dNHWC``: max pooling for channels_last activations with 1-byte window codes.

PyTorch's ``max_pool2d_with_indices`` saves an int64 index per output element (ResNet-50 stem:
205 MB written in forward, read in backward -- 8x the pooled tensor) and its backward scatters
into a zero-filled gradient.  ``csrc/kernels/pool.hip`` saves the in-window argmax as one byte
and GATHERS in backward (every input element sums the gradients of the windows whose code
points at it: no zero fill, no atomics, deterministic).  Same semantics as ``nn.MaxPool2d``
(first maximum wins, NaN propagates, implicit -inf padding); other layouts / dtypes, dilation,
``ceil_mode`` and ``return_indices`` take the PyTorch path.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        y, code = _native.lib().maxpool_fwd(x, k, s, pad)
        ctx.save_for_backward(code)
        ctx.geom = (x.shape[2], x.shape[3], k, s, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (code,) = ctx.saved_tensors
        H, W, k, s, pad = ctx.geom
        if not dy.is_contiguous(memory_format=torch.channels_last) or dy.data_ptr() % 16:
            dy = dy.contiguous(memory_format=torch.channels_last)
            if dy.data_ptr() % 16:
                dy = dy.clone(memory_format=torch.channels_last)
        return _native.lib().maxpool_bwd(dy, code, H, W, k, s, pad), None, None, None


class MaxPool2dNHWC(nn.MaxPool2d):
    """Drop-in ``nn.MaxPool2d`` (square kernel / stride / padding) with the native NHWC kernels."""

    def _native_ok(self, x: torch.Tensor) -> bool:
        k, s, p, d = _pair(self.kernel_size), _pair(self.stride or self.kernel_size), _pair(self.padding), _pair(self.dilation)
        return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16)
                and _native.native_on(x.device) and x.is_contiguous(memory_format=torch.channels_last)
                and x.shape[1] % 8 == 0 and x.data_ptr() % 16 == 0 and x.numel() > 0
                and k[0] == k[1] and s[0] == s[1] and p[0] == p[1] and d == (1, 1) and k[0] <= 15
                and 2 * p[0] <= k[0] and not self.ceil_mode and not self.return_indices
                and x.shape[2] + 2 * p[0] >= k[0] and x.shape[3] + 2 * p[0] >= k[0])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._native_ok(x):
            k, s, p = _pair(self.kernel_size)[0], _pair(self.stride or self.kernel_size)[0], _pair(self.padding)[0]
            return _MaxPoolFn.apply(x, k, s, p)
        return super().forward(x)


class _GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        ctx.dtype = x.dtype
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, dy):
        dy = dy.to(ctx.dtype).contiguous()
        if dy.data_ptr() % 16:
            dy = dy.clone()
        return _native.lib().gap_bwd(dy, ctx.hw[0], ctx.hw[1])


class GlobalAvgPoolFlat(nn.Module):
    """``flatten(adaptive_avg_pool2d(x, 1), 1)`` with a native backward for channels_last x: the
    gradient is one broadcast pass (PyTorch's expand + div runs two non-vectorised channels_last
    kernels, ~26 us for the ResNet-50 head at batch 32)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16) and _native.native_on(x.device)
                and x.is_contiguous(memory_format=torch.channels_last) and x.shape[1] % 8 == 0 and x.numel() > 0):
            return _GapFn.apply(x)
        return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
