"""SketchML-style quantile sketch (Jiang et al., SIGMOD 2018) -- the TF-only ``Sketch``.

Reference: /root/reference/grace_dl/tensorflow/compressor/sketch.py:6-39 -- q+1 linear
quantile edges of x (tfp.stats.quantiles), bin of every element (tfp find_bins), payload =
(bin uint8 -- uint16 when q >= 256 -- , mean of every bin); decompress = means[bin].

Here per segment: edges from torch.quantile (linear interpolation, as the reference), bins by
searchsorted clamped to [0, q-1] (values equal to the last edge go to the last bin), bin means
by index_add.  Payload [bins uint8/int16 | means fp32 (q per segment)].  On the GPU the edges of
ALL segments come from one segmented sort, and bucketisation + per-bin sums/counts
(csrc/kernels/cast_sketch.hip) and the W-rank decode are single passes.
"""
from __future__ import annotations

import torch

from ..ops import _native
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


def segmented_quantile_edges(x: torch.Tensor, lay, q: int) -> torch.Tensor:
    """[n_seg, q+1] linear-interpolation quantile edges of every segment from ONE sort of the
    bucket (keys = segment id << 32 | order-preserving float bits)."""
    dev = x.device
    seg_id = lay.cached(dev, "seg_id", lambda: torch.repeat_interleave(
        torch.arange(lay.n_seg, device=dev), lay.numels_t(dev, torch.int64)))
    u = x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    ordered = torch.where(u >= 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    order = torch.sort((seg_id << 32) | ordered).indices
    sx = x[order]
    offs = lay.offsets_t(dev, torch.float64)[:-1]
    n = lay.numels_t(dev, torch.float64)
    probs = torch.linspace(0, 1, q + 1, device=dev, dtype=torch.float64)
    pos = probs[None, :] * (n[:, None] - 1).clamp_min(0)
    lo, hi = pos.floor(), pos.ceil()
    w = (pos - lo).float()
    a = sx[(offs[:, None] + lo).long()]
    b = sx[(offs[:, None] + hi).long()]
    return (a * (1 - w) + b * w).contiguous()


_QSEL_CHUNK = 65536  # elements per workgroup of the selection passes (LDS setup amortised)
_CODEC_CHUNK = 32768  # encode / decode: per-workgroup LDS bin tables amortised over 32K elements


def _qsel_tables(lay, q: int, dev: torch.device):
    """Per-layout tables of the native selection: the sorted distinct ranks floor/ceil(j (n-1)/q)
    of every segment, the positions of each edge's two ranks among them, the interpolation
    weights (float64 positions rounded to fp32 exactly as ``segmented_quantile_edges``) and the
    zero-initialised histograms / state the kernels leave clean after every call."""
    def build():
        n = torch.tensor(lay.numels, dtype=torch.float64)
        probs = torch.linspace(0, 1, q + 1, dtype=torch.float64)
        pos = probs[None, :] * (n[:, None] - 1).clamp_min(0)
        lo, hi = pos.floor(), pos.ceil()
        w = (pos - lo).float()
        per = []
        for i in range(lay.n_seg):
            per.append(sorted(set(lo[i].long().tolist()) | set(hi[i].long().tolist())) if lay.numels[i] else [])
        ms = max(1, max(len(r) for r in per))
        if ms > 256:
            return None
        ranks = torch.zeros(lay.n_seg, ms, dtype=torch.int32)
        lo_idx = torch.zeros(lay.n_seg, q + 1, dtype=torch.int32)
        hi_idx = torch.zeros(lay.n_seg, q + 1, dtype=torch.int32)
        for i, r in enumerate(per):
            if not r:
                continue
            ranks[i, :len(r)] = torch.tensor(r, dtype=torch.int32)
            where = {v: j for j, v in enumerate(r)}
            lo_idx[i] = torch.tensor([where[int(v)] for v in lo[i].tolist()], dtype=torch.int32)
            hi_idx[i] = torch.tensor([where[int(v)] for v in hi[i].tolist()], dtype=torch.int32)
        z = lambda *shape: torch.zeros(*shape, dtype=torch.int32, device=dev)
        return {"max_slots": ms, "ranks": ranks.to(dev), "nrank": torch.tensor([len(r) for r in per], dtype=torch.int32,
                                                                               device=dev),
                "lo_idx": lo_idx.to(dev), "hi_idx": hi_idx.to(dev), "w": w.contiguous().to(dev),
                "h0": z(lay.n_seg * 2048), "h": z(lay.n_seg * ms * 128), "st_pfx": z(lay.n_seg * ms),
                "st_rank": z(lay.n_seg * ms), "slot": z(lay.n_seg * ms), "uniq": z(lay.n_seg * ms),
                "nuniq": z(lay.n_seg)}
    return lay.cached(dev, f"qsel:{q}", build)


def native_quantile_edges(x: torch.Tensor, lay, q: int):
    """[n_seg, q+1] edges from the HIP multi-rank radix select (csrc/kernels/quantile.hip), or
    None when the layout needs more than 256 distinct ranks per segment (q > 127)."""
    tb = _qsel_tables(lay, q, x.device)
    if tb is None:
        return None
    ct = lay.device_tables(x.device, _QSEL_CHUNK)
    edges = torch.empty(lay.n_seg, q + 1, device=x.device)
    _native.lib().quantile_select(x, ct["seg"], ct["begin"], ct["end"], lay.n_seg, tb["max_slots"], tb["ranks"],
                                  tb["nrank"], tb["h0"], tb["h"], tb["st_pfx"], tb["st_rank"], tb["slot"],
                                  tb["uniq"], tb["nuniq"], q, tb["lo_idx"], tb["hi_idx"], tb["w"], edges)
    return edges


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
        if _native.use_native(x) and q <= 1024:
            edges = native_quantile_edges(x, lay, q)
            if edges is None:
                edges = segmented_quantile_edges(x, lay, q)
            sums = torch.zeros(lay.n_seg * q, device=x.device)
            cnts = torch.zeros(lay.n_seg * q, device=x.device)
            t = lay.device_tables(x.device, _CODEC_CHUNK)
            _native.lib().sketch_encode(x, edges, q, bins, sums, cnts, t["seg"], t["begin"], t["end"])
            torch.where(cnts > 0, sums / cnts.clamp_min(1), torch.zeros_like(sums), out=means)
            return [bins, means], ctx
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
        if _native.use_native(per_rank[0][0]):
            base, stride, offs = self.rows(per_rank)
            out = self.out_buffer(ctx, base.device)
            t = lay.device_tables(base.device, _CODEC_CHUNK)
            _native.lib().sketch_decode(base, stride, offs[0], offs[1], q, per_rank[0][0].element_size(), n_ranks,
                                        scale, out, t["seg"], t["begin"], t["end"], lay.n_seg)
            return self.finish(out, ctx)
        out = self.out_buffer(ctx, per_rank[0][0].device, zero=True)
        seg_id = torch.repeat_interleave(torch.arange(lay.n_seg, device=out.device),
                                         lay.numels_t(out.device, torch.int64))
        for bins, means in per_rank:
            b = bins.long()
            if bins.dtype == torch.int16:
                b = b & 0xFFFF
            out += means[seg_id * q + b]
        if scale != 1.0:
            out *= scale
        return self.finish(out, ctx)
