"""SketchML-style quantile sketch (Jiang et al., SIGMOD 2018) -- the TF-only ``Sketch``.

Reference: /root/reference/grace_dl/tensorflow/compressor/sketch.py:6-39 -- q+1 linear
quantile edges of x (tfp.stats.quantiles), bin of every element (tfp find_bins), payload =
(bin uint8 -- uint16 when q >= 256 -- , mean of every bin); decompress = means[bin].

Here per segment: edges from torch.quantile (linear interpolation, as the reference), bins by
searchsorted clamped to [0, q-1] (values equal to the last edge go to the last bin), bin means
by index_add.  Payload [bins uint8/int16 | means fp32 (q per segment)].  PyTorch-ROCm ops (no
dedicated HIP kernel yet).
"""
from __future__ import annotations

import torch

from ._base import BucketCompressor


def _quantiles(seg: torch.Tensor, probs: torch.Tensor) -> torch.Tensor:
    """Linear-interpolation quantiles (tfp.stats.quantiles(..., interpolation='linear')) via one
    sort -- torch.quantile rejects inputs above 2^24 elements."""
    srt = torch.sort(seg).values
    pos = probs * (seg.numel() - 1)
    lo = pos.floor().long()
    hi = pos.ceil().long()
    w = pos - lo.float()
    return srt[lo] * (1 - w) + srt[hi] * w


class SketchCompressor(BucketCompressor):
    reduce_by_allgather = True
    allreduce_compatible = True

    def __init__(self, quantiles: int = 64):
        super().__init__()
        self.quantiles = int(quantiles)

    def compress(self, tensor, name):
        ctx = self.ctx(tensor, name)
        x = self.flat(tensor)
        lay, q = ctx.layout, self.quantiles
        bdt = torch.uint8 if q < 256 else torch.int16
        bins, means = self.payload(x.device, [(bdt, (lay.total,)), (torch.float32, (q * lay.n_seg,))])
        probs = torch.linspace(0, 1, q + 1, device=x.device)
        for i, o, n in lay.segments():
            seg = x[o:o + n]
            edges = _quantiles(seg, probs) if n > 1 else seg.repeat(q + 1)
            b = (torch.searchsorted(edges, seg.contiguous(), right=True) - 1).clamp(0, q - 1)
            s = torch.zeros(q, device=x.device).index_add_(0, b, seg)
            c = torch.zeros(q, device=x.device).index_add_(0, b, torch.ones_like(seg))
            means[i * q:(i + 1) * q] = torch.where(c > 0, s / c.clamp_min(1), torch.zeros_like(s))
            bins[o:o + n] = b.to(bdt)
        return [bins, means], ctx

    def decompress_aggregate_impl(self, per_rank, ctx, n_ranks, scale):
        lay, q = ctx.layout, self.quantiles
        out = self.out_buffer(ctx, per_rank[0][0].device, zero=True)
        seg_id = torch.repeat_interleave(torch.arange(lay.n_seg, device=out.device),
                                         torch.tensor(lay.numels, device=out.device))
        for bins, means in per_rank:
            b = bins.long()
            if bins.dtype == torch.int16:
                b = b & 0xFFFF
            out += means[seg_id * q + b]
        if scale != 1.0:
            out *= scale
        return self.finish(out, ctx)
