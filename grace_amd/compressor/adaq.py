"""AdaComp-style two-sided quantization (Dryden et al., MLHPC 2016) -- the TF-only ``Adaq``.

Reference: /root/reference/grace_dl/tensorflow/compressor/adaq.py:6-93 -- for the positive and
the negative entries separately: estimate a threshold from a 1% sample so that about
``ratio`` of that side's entries pass, refine it (x1.25 if > 1.25*target, else x0.9, while the
count is outside [0.8, 1.25]*target, at most 20 times; if nothing passes lower it by 0.8),
then send only the MEAN of the selected values and their indices:
``[plus_mean, minus_mean, n_plus, plus_idx..., minus_idx...]`` as one int32 tensor.
Decompress writes plus_mean / minus_mean at the indices.

MI355X (csrc/kernels/adaq.hip): every segment of a bucket and both sides at once, on the
device -- Philox 1% sample, the segmented radix select of topk.hip for the initial thresholds,
the refinement loop with both sides counted per pass over the bucket, ordered compaction of the
indices and deterministic per-group means.  The payload has a FIXED index capacity (default 2 x
the summed targets) and the per-group counts in-band, so nothing is read back to the host and the
exchange is graph-capturable; the decoder scans the counts on the device.  The PyTorch path
(per segment, torch RNG, sampling among the side's entries exactly as the reference) is the
CPU oracle.  Payload [means fp32 (+,- per segment) | counts int32 (+,- per segment) | indices
int32].  A side with no entries sends mean 0 and no index (the reference computes the mean of
an empty set -> NaN).  Entries selected past the capacity are not sent (their group's mean still
covers them).
"""
from __future__ import annotations

import math

import torch

from ..ops import _native
from ..ops import segstats as S
from ..ops import topk as K
from ..ops.layout import SegmentLayout
from ._base import BucketCompressor


def _side(vals_abs: torch.Tensor, ratio: float, gen) -> torch.Tensor:
    """Boolean selection over one side's |values| (reference quan(), adaq.py:16-51)."""
    n = vals_abs.numel()
    if n == 0:
        return torch.zeros(0, dtype=torch.bool, device=vals_abs.device)
    ns = max(1, math.ceil(n * 0.01))
    k = max(1, math.ceil(n * 0.01 * ratio))
    pos = (torch.rand(ns, generator=gen, device=vals_abs.device) * n).long().clamp_max(n - 1)
    thr = torch.topk(vals_abs[pos], min(k, ns)).values.min()
    target = math.ceil(n * ratio)
    mask = vals_abs > thr
    sel = int(mask.sum())
    it = 0
    while (sel > 1.25 * target or sel < 0.8 * target) and it < 20:
        thr = thr * 1.25 if sel > 1.25 * target else thr * 0.9
        mask = vals_abs >= thr
        sel = int(mask.sum())
        it += 1
    if sel < 1:
        thr = thr * 0.8
    return vals_abs > thr


class AdaqCompressor(BucketCompressor):
    def __init__(self, compress_ratio: float = 0.01, capacity: float = 2.0):
        super().__init__(tensors_size_are_same=True)  # fixed-capacity payload, counts in-band
        self.compress_ratio = compress_ratio
        self.capacity = capacity

    def _cap(self, lay) -> int:
        """Index capacity: ``capacity`` x the summed per-side targets (<= ceil(n_i * ratio) + 1
        per side), at most the bucket."""
        tgt = sum(n * self.compress_ratio + 2 for n in lay.numels if n > 0)
        return max(1, min(lay.total, int(math.ceil(self.capacity * tgt))))

    max_iters = 20

    def _native_compress(self, x, lay, name):
        C = _native.lib()
        dev = x.device

        def build():
            ns = [max(1, math.ceil(n * 0.01)) if n > 0 else 0 for n in lay.numels]
            off = [0]
            for v in ns:
                off.append(off[-1] + v)
            gl = SegmentLayout(tuple(v for v in ns for _ in (0, 1)), tuple((v,) for v in ns for _ in (0, 1)))
            ng = 2 * lay.n_seg
            i32 = dict(dtype=torch.int32, device=dev)
            f32 = dict(dtype=torch.float32, device=dev)
            return {
                "samp_off": torch.tensor(off, dtype=torch.int64, device=dev),
                "glay": gl, "gt": gl.device_tables(dev),
                "samples": torch.empty(max(1, gl.total), **f32),
                "count": torch.empty(ng, **i32), "target": torch.empty(ng, **f32), "kseg": torch.empty(ng, **i32),
                "fallback": torch.empty(ng, **f32), "thr": torch.empty(ng, **f32), "done": torch.empty(ng, **i32),
                "state": torch.zeros(2 * ng, **i32), "hist": torch.zeros(ng * 2048, **i32),
                "goff": torch.empty(ng + 1, **i32), "cursor": torch.empty(ng, **i32),
            }

        ws = lay.cached(dev, f"adaq_ws:{self.compress_ratio}", build)
        t = lay.device_tables(dev)
        seed, step = self.next_rng(name, dev)
        sd = seed - (1 << 64) if seed >= (1 << 63) else seed
        stats = S.segment_stats(x, lay)
        C.adaq_sample(x, t["offsets"], ws["samp_off"], sd, step, ws["samples"][: ws["glay"].total])
        C.adaq_prepare(x, t["offsets"], ws["samp_off"], stats, self.compress_ratio, ws["count"], ws["target"],
                       ws["kseg"], ws["fallback"], ws["thr"], ws["done"], t["seg"], t["begin"], t["end"])
        gt = ws["gt"]
        smp = ws["samples"][: ws["glay"].total]
        C.topk_select(smp, None, smp, 1.0, 1.0, 0, gt["seg"], gt["begin"], gt["end"], ws["kseg"], ws["state"],
                      ws["hist"])
        C.adaq_refine(x, ws["state"], ws["fallback"], ws["target"], self.max_iters, ws["thr"], ws["count"],
                      ws["done"], t["seg"], t["begin"], t["end"])
        C.adaq_offsets(ws["count"], ws["goff"], ws["cursor"])
        m, cnt, ix = self.payload(dev, [(torch.float32, (2 * lay.n_seg,)), (torch.int32, (2 * lay.n_seg,)),
                                        (torch.int32, (self._cap(lay),))])
        psum = torch.empty(max(1, 2 * t["n_chunks"]), dtype=torch.float64, device=dev)
        C.adaq_compact(x, ws["thr"], ws["goff"], ws["cursor"], ix, psum, m, cnt, t["seg"], t["begin"], t["end"],
                       t["seg_chunk_begin"])
        return [m, cnt, ix]

    def compress(self, tensor, name):
        ctx = self.ctx(tensor, name)
        x = self.flat(tensor)
        lay = ctx.layout
        if _native.use_native(x):
            return self._native_compress(x, lay, name), ctx
        gen = torch.Generator(device=x.device)
        gen.manual_seed(self.next_seed(name) & 0x7FFFFFFFFFFFFFFF)
        means = torch.zeros(2 * lay.n_seg, dtype=torch.float32, device=x.device)
        counts = torch.zeros(2 * lay.n_seg, dtype=torch.int32)
        idx_all = []
        for i, o, n in lay.segments():
            seg = x[o:o + n]
            for side in (0, 1):  # 0: positive entries, 1: negative entries
                (sidx,) = torch.where(seg > 0 if side == 0 else seg < 0)
                chosen = sidx[_side(seg[sidx].abs(), self.compress_ratio, gen)]
                if chosen.numel():
                    means[2 * i + side] = seg[chosen].mean()
                counts[2 * i + side] = chosen.numel()
                idx_all.append((chosen + o).to(torch.int32))
        idx = torch.cat(idx_all) if idx_all else torch.empty(0, dtype=torch.int32, device=x.device)
        cap = self._cap(lay)
        m, cnt, ix = self.payload(x.device, [(torch.float32, (2 * lay.n_seg,)), (torch.int32, (2 * lay.n_seg,)),
                                             (torch.int32, (cap,))])
        # groups back to back; the in-band counts are the entries inside the capacity
        goff = torch.cumsum(counts.long(), 0) - counts.long()
        counts = (torch.clamp(cap - goff, min=0)).minimum(counts.long()).to(torch.int32)
        m.copy_(means)
        cnt.copy_(counts)
        ix.zero_()
        k = min(cap, idx.numel())
        ix[:k] = idx[:k]
        return [m, cnt, ix], ctx

    def decompress_aggregate_impl(self, per_rank, ctx, n_ranks, scale):
        dev = per_rank[0][0].device
        out = self.out_buffer(ctx, dev, zero=True)
        if _native.use_native(out):
            C = _native.lib()
            ws = ctx.layout.cached(dev, "adaq_dec", lambda: torch.empty(2 * ctx.layout.n_seg + 1, dtype=torch.int32,
                                                                        device=dev))
            for means, counts, idx in per_rank:  # rank order: identical on every rank
                C.adaq_decode(means, counts, idx, ws, out, scale)
            return self.finish(out, ctx)
        for means, counts, idx in per_rank:
            reps = counts.to(device=means.device, dtype=torch.int64)
            v = torch.repeat_interleave(means, reps)  # [plus_0.., minus_0.., plus_1.., ...]
            K.scatter_add(v, idx[: v.numel()], out, scale, accumulate=True)
        return self.finish(out, ctx)
