"""Per-segment statistics of a flat bucket in one pass (native: csrc/kernels/segstats.hip).

Columns of the returned ``[n_seg, 6]`` fp32 tensor:
SUM, SUMSQ, ABSMAX, ABSSUM, NEGSUM, NEGCNT.
"""
from __future__ import annotations

import torch

from . import _native
from .layout import SegmentLayout

SUM, SUMSQ, ABSMAX, ABSSUM, NEGSUM, NEGCNT = range(6)
NSTAT = 6


def segment_stats(x: torch.Tensor, layout: SegmentLayout, r: torch.Tensor | None = None, r_valid: bool = False,
                  beta: float = 1.0, gamma: float = 1.0, xout: torch.Tensor | None = None) -> torch.Tensor:
    """Statistics of x (or of the compensated x = beta*r + gamma*g when ``r_valid``; the
    compensated values are stored into ``xout`` when given)."""
    assert x.dim() == 1 and x.numel() == layout.total
    mode = 1 if (r is not None and r_valid) else 0
    if _native.use_native(x):
        t = layout.device_tables(x.device)
        part = layout.cached(x.device, "segstats_part",
                             lambda: torch.empty(max(1, t["n_chunks"]) * NSTAT, dtype=torch.float64, device=x.device))
        stats = torch.empty(layout.n_seg, NSTAT, dtype=torch.float32, device=x.device)  # fold writes all
        _native.lib().segment_stats(x, r if mode else None, mode, beta, gamma, xout, t["seg"], t["begin"], t["end"],
                                    t["seg_chunk_begin"], part, stats)
        return stats
    if mode == 1:
        x = beta * r + gamma * x
    if xout is not None:
        if xout.data_ptr() != x.data_ptr():
            xout.copy_(x)
        x = xout
    out = torch.zeros(layout.n_seg, NSTAT, dtype=torch.float64)
    for i, o, n in layout.segments():
        if n == 0:
            continue
        s = x[o:o + n].double()
        neg = s[s < 0]
        out[i, SUM] = s.sum()
        out[i, SUMSQ] = (s * s).sum()
        out[i, ABSMAX] = s.abs().max()
        out[i, ABSSUM] = s.abs().sum()
        out[i, NEGSUM] = neg.sum()
        out[i, NEGCNT] = neg.numel()
    return out.float().to(x.device)


def expand(per_seg: torch.Tensor, layout: SegmentLayout) -> torch.Tensor:
    """Broadcast a per-segment value to every element (torch path helper)."""
    reps = layout.numels_t(per_seg.device, torch.int64)
    return torch.repeat_interleave(per_seg, reps)
