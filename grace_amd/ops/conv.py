"""fp32 1x1 convolutions of channels_last activations on the hand-written f32 MFMA GEMM.

A 1x1 stride-1 convolution over a channels_last activation is a plain GEMM over its
[M = N*H*W, C] view (no im2col), so all three of its products run on
``csrc/kernels/gemm_f32.hip`` (``v_mfma_f32_32x32x2_f32``, exact fp32):

    forward      Y[M, Cout]    = X[M, Cin] . W[Cout, Cin]^T
    data grad    dX[M, Cin]    = dY[M, Cout] . W[Cout, Cin]
    weight grad  dW[Cout, Cin] = dY^T . X           (split-K over M, f32 atomics)

``Conv1x1F32`` is a drop-in ``nn.Conv2d`` subclass (same parameters / state_dict) used by the
ResNet bottlenecks; it falls back to ``F.conv2d`` whenever the fast path does not apply (CPU,
bf16/autocast, non-channels_last input, odd channel counts, stride/padding/groups/bias).

Opt-in (``GRACE_CONV_MFMA=1`` or ``set_enabled(True)``): measured per layer on ResNet-50 b32
(profiles/r2_conv_fp32_mfma_vs_miopen.txt) the kernel is within ~10 % of MIOpen's tuned
implicit-GEMM solvers (fwd+bwd of the 1x1 stride-1 layers 4.87 vs 4.47 ms per step), ahead on
some backward shapes and behind on the memory-bound small-K forwards, so MIOpen stays the
default conv path.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native

_TARGET_BLOCKS = 512  # >> 256 CUs


def _splits(m: int, n: int, k: int) -> int:
    tm = (m + 127) // 128 if m > 64 else 1
    tn = (n + 127) // 128 if n > 64 or m <= 64 else 1
    tiles = tm * tn
    return max(1, min(math.ceil(_TARGET_BLOCKS / tiles), k // 256))


def gemm(a, a_kc, lda, b, b_kc, ldb, c, ldc, m, n, k, splits=1):
    """C[m, n] = sum_k A(m, k) B(n, k) (see csrc/kernels/gemm_f32.hip); splits=0: split-K chosen by
    the launcher when the output has too few tiles to fill the chip (needs a dense C)."""
    _native.lib().gemm_f32(a, a_kc, lda, b, b_kc, ldb, c, ldc, m, n, k, splits)


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        nb, cin, h, w = x.shape
        cout = weight.shape[0]
        m = nb * h * w
        wt = weight.reshape(cout, cin)
        if not wt.is_contiguous():
            wt = wt.contiguous()
        y = torch.empty((nb, cout, h, w), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
        gemm(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 0)
        ctx.save_for_backward(x, wt)
        ctx.wshape = weight.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        nb, cin, h, w = x.shape
        cout = wt.shape[0]
        m = nb * h * w
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            gemm(dy, True, cout, wt, False, cin, dx, cin, m, cin, cout, 0)
        if ctx.needs_input_grad[1]:
            dw = torch.empty((cout, cin), device=x.device, dtype=torch.float32)
            gemm(dy, False, cout, x, False, cin, dw, cin, cout, cin, m, _splits(cout, cin, m))
            dw = dw.view(ctx.wshape)
        return dx, dw


_ENABLED = os.environ.get("GRACE_CONV_MFMA", "0") == "1"


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def fast_ok(x: torch.Tensor, conv: nn.Conv2d, force: bool = False) -> bool:
    if not (_ENABLED or force):
        return False
    if not (x.is_cuda and x.dtype == torch.float32 and conv.weight.dtype == torch.float32):
        return False
    if torch.is_autocast_enabled() or not _native.native_on(x.device):
        return False
    if conv.kernel_size != (1, 1) or conv.stride != (1, 1) or conv.padding != (0, 0) or conv.groups != 1 \
            or conv.dilation != (1, 1) or conv.bias is not None:
        return False
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16:
        return False
    cin, cout = conv.in_channels, conv.out_channels
    return cin % 4 == 0 and cout % 4 == 0 and x.shape[0] * x.shape[2] * x.shape[3] % 4 == 0


class Conv1x1F32(nn.Conv2d):
    """``nn.Conv2d(cin, cout, 1, bias=False)`` whose fp32 channels_last path runs on the f32 MFMA GEMM."""

    def __init__(self, cin: int, cout: int, **kw):
        super().__init__(cin, cout, 1, bias=False, **kw)

    def forward(self, x):
        if fast_ok(x, self):
            return _Conv1x1Fn.apply(x, self.weight)
        return super().forward(x)
