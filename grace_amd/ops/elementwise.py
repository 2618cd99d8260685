"""Elementwise helpers used by the memories (native: csrc/kernels/ef.hip)."""
from __future__ import annotations

import torch

from . import _native


def axpby(x: torch.Tensor, y: torch.Tensor, a: float, b: float, out: torch.Tensor | None = None) -> torch.Tensor:
    """out = a*x + b*y (fp32, one fused pass)."""
    if out is None:
        out = torch.empty_like(y)
    if (_native.use_native(y) and y.dtype == torch.float32 and x.dtype == torch.float32
            and x.is_contiguous() and y.is_contiguous() and out.is_contiguous()):
        _native.lib().axpby(x.reshape(-1), y.reshape(-1), out.reshape(-1), a, b)
        return out
    torch.add(x * a, y, alpha=b, out=out) if a != 1.0 else torch.add(x, y, alpha=b, out=out)
    return out


def scale_(x: torch.Tensor, s: float) -> torch.Tensor:
    if _native.use_native(x) and x.dtype == torch.float32 and x.is_contiguous():
        _native.lib().scale_(x.view(-1), s)
        return x
    return x.mul_(s)
