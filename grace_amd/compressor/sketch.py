"""SketchML-style quantile sketch (Jiang et al., SIGMOD 2018) -- the TF-only ``Sketch``.

Reference: /root/reference/grace_dl/tensorflow/compressor/sketch.py:6-39 -- q+1 linear
quantile edges of x (tfp.stats.quantiles), bin of every element (tfp find_bins), payload =
(bin uint8 -- uint16 when q >= 256 -- , mean of every bin); decompress = means[bin].

Here per segment: edges from torch.quantile (linear interpolation, as the reference), bins by
searchsorted clamped to [0, q-1] (values equal to the last edge go to the last bin), bin means
by index_add.  Payload [bins uint8/int16 | means fp32 (q per segment)].  On the GPU the edges of
ALL segments come from the native segmented multi-rank radix select (csrc/kernels/quantile.hip;
any q up to 65535, the reference's uint16 range: q >= 128 runs it in batches of 256 ranks per
segment), and bucketisation + per-bin sums/counts (csrc/kernels/cast_sketch.hip: per-wave LDS bin
tables up to q = 1024, global fixed-point accumulators above) and the W-rank decode are single
passes -- no sort on the GPU path, graph-capturable for every q.
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


import os as _os

# elements per workgroup of the selection passes (LDS setup amortised) and of encode / decode
# (per-workgroup LDS bin tables amortised); env-tunable for sweeps on the GPU box
# (< 65536: the selection histograms pack two 16-bit bin counts per LDS word)
_QSEL_CHUNK = min(int(_os.environ.get("GRACE_QSEL_CHUNK", 32768)), 65535)
_CODEC_CHUNK = int(_os.environ.get("GRACE_CODEC_CHUNK", 8192))


_QSEL_MAX_RANKS = 256  # distinct target ranks per segment one selection batch resolves


def _rank_plan(lay, q: int):
    """Per segment: the sorted distinct ranks floor/ceil(j (n-1)/q) and each edge's two positions
    among them, plus the interpolation weights (float64 positions rounded to fp32 exactly as
    ``segmented_quantile_edges``)."""
    n = torch.tensor(lay.numels, dtype=torch.float64)
    probs = torch.linspace(0, 1, q + 1, dtype=torch.float64)
    pos = probs[None, :] * (n[:, None] - 1).clamp_min(0)
    lo, hi = pos.floor(), pos.ceil()
    w = (pos - lo).float()
    per, lo_idx, hi_idx = [], torch.zeros(lay.n_seg, q + 1, dtype=torch.int32), torch.zeros(lay.n_seg, q + 1,
                                                                                            dtype=torch.int32)
    for i in range(lay.n_seg):
        r = sorted(set(lo[i].long().tolist()) | set(hi[i].long().tolist())) if lay.numels[i] else []
        per.append(r)
        if r:
            where = {v: j for j, v in enumerate(r)}
            lo_idx[i] = torch.tensor([where[int(v)] for v in lo[i].tolist()], dtype=torch.int32)
            hi_idx[i] = torch.tensor([where[int(v)] for v in hi[i].tolist()], dtype=torch.int32)
    return per, lo_idx, hi_idx, w


def _batch_tables(lay, per, dev, lo_idx=None, hi_idx=None, w=None, q=None):
    """Device tables of one selection batch (<= 256 distinct ranks per segment).  Without
    lo/hi/w the batch emits the VALUES of its ranks (edge j = rank j: lo = hi = j, w = 0)."""
    ms = max(1, max(len(r) for r in per))
    ranks = torch.zeros(lay.n_seg, ms, dtype=torch.int32)
    for i, r in enumerate(per):
        if r:
            ranks[i, :len(r)] = torch.tensor(r, dtype=torch.int32)
    if lo_idx is None:
        nq = ms - 1
        ident = torch.stack([torch.clamp(torch.arange(ms), max=max(0, len(r) - 1)) for r in per]).to(torch.int32)
        lo_idx, hi_idx, w, q = ident, ident, torch.zeros(lay.n_seg, ms), nq
    z = lambda *shape: torch.zeros(*shape, dtype=torch.int32, device=dev)
    return {"max_slots": ms, "q": q, "ranks": ranks.to(dev),
            "nrank": torch.tensor([len(r) for r in per], dtype=torch.int32, device=dev),
            "lo_idx": lo_idx.contiguous().to(dev), "hi_idx": hi_idx.contiguous().to(dev), "w": w.contiguous().to(dev),
            "h0": z(lay.n_seg * 2048), "h": z(lay.n_seg * ms * 128), "st_pfx": z(lay.n_seg * ms),
            "st_rank": z(lay.n_seg * ms), "slot": z(lay.n_seg * ms), "uniq": z(lay.n_seg * ms),
            "nuniq": z(lay.n_seg)}


def _qsel_tables(lay, q: int, dev: torch.device):
    """Per-layout selection plan.  q <= 127 (<= 256 distinct ranks per segment): ONE batch that
    emits the interpolated edges directly.  Larger q: the distinct ranks are split into batches
    of <= 256 per segment; each batch emits the VALUES of its ranks, and the edges are
    interpolated from them (same unfused fp32 mul/add rounding as the kernel and the sort path).
    The workspaces are zero-initialised; the kernels leave them clean after every call."""
    def build():
        per, lo_idx, hi_idx, w = _rank_plan(lay, q)
        ms = max(1, max(len(r) for r in per))
        if ms <= _QSEL_MAX_RANKS:
            return {"direct": _batch_tables(lay, per, dev, lo_idx, hi_idx, w, q)}
        nb = -(-ms // _QSEL_MAX_RANKS)
        batches = [_batch_tables(lay, [r[b * _QSEL_MAX_RANKS:(b + 1) * _QSEL_MAX_RANKS] for r in per], dev)
                   for b in range(nb)]
        return {"batches": batches, "ms": ms, "lo_idx": lo_idx.long().to(dev), "hi_idx": hi_idx.long().to(dev),
                "w": w.to(dev)}
    return lay.cached(dev, f"qsel:{q}", build)


def _run_select(x, lay, ct, tb, out):
    _native.lib().quantile_select(x, ct["seg"], ct["begin"], ct["end"], lay.n_seg, tb["max_slots"], tb["ranks"],
                                  tb["nrank"], tb["h0"], tb["h"], tb["st_pfx"], tb["st_rank"], tb["slot"],
                                  tb["uniq"], tb["nuniq"], tb["q"], tb["lo_idx"], tb["hi_idx"], tb["w"], out)


def native_quantile_edges(x: torch.Tensor, lay, q: int):
    """[n_seg, q+1] edges from the HIP multi-rank radix select (csrc/kernels/quantile.hip), for
    any q: one batch of <= 256 distinct ranks per segment, or several (q >= 128) whose selected
    values are then interpolated.  Bit-identical to ``segmented_quantile_edges``; no sort, no
    host read (graph-capturable)."""
    tb = _qsel_tables(lay, q, x.device)
    ct = lay.device_tables(x.device, _QSEL_CHUNK)
    if "direct" in tb:
        edges = torch.empty(lay.n_seg, q + 1, device=x.device)
        _run_select(x, lay, ct, tb["direct"], edges)
        return edges
    vals = torch.empty(lay.n_seg, len(tb["batches"]) * _QSEL_MAX_RANKS, device=x.device)
    for b, bt in enumerate(tb["batches"]):
        vb = torch.empty(lay.n_seg, bt["max_slots"], device=x.device)
        _run_select(x, lay, ct, bt, vb)
        vals[:, b * _QSEL_MAX_RANKS:b * _QSEL_MAX_RANKS + bt["max_slots"]] = vb
    a = vals.gather(1, tb["lo_idx"])
    c = vals.gather(1, tb["hi_idx"])
    w = tb["w"]
    return a * (1 - w) + c * w


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
        if _native.use_native(x) and q <= 65535:
            edges = native_quantile_edges(x, lay, q)
            t = lay.device_tables(x.device, _CODEC_CHUNK)
            # persistent, self-cleaning totals: the segment's last encode block writes the means and
            # re-zeroes them (no fills, no elementwise mean kernels)
            # (bin sums in int64 fixed point: csrc/kernels/cast_sketch.hip)
            ws = lay.cached(x.device, f"sketch_ws:{q}", lambda: {
                "sums": torch.zeros(lay.n_seg * q, dtype=torch.int64, device=x.device),
                "cnts": torch.zeros(lay.n_seg * q, dtype=torch.int32, device=x.device),
                "arrive": torch.zeros(lay.n_seg, dtype=torch.int32, device=x.device)})
            _native.lib().sketch_encode(x, edges, q, bins, ws["sums"], ws["cnts"], t["seg"], t["begin"], t["end"],
                                        ws["arrive"], t["seg_chunk_begin"], means)
            return [bins, means], ctx
        # edges at float64 quantile positions j (n-1) / q (the native select's exact ranks and
        # weights: fp32 positions mis-round for q not a power of two)
        all_edges = segmented_quantile_edges(x, lay, q) if lay.total else None
        for i, o, n in lay.segments():
            seg = x[o:o + n]
            edges = all_edges[i].contiguous()
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
