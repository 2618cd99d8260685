"""DGC threshold selection (native: csrc/kernels/dgc.hip + the segmented radix select)."""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch

from . import _native
from .layout import SegmentLayout
from .topk import _workspace as _topk_ws


def _sizes(layout: SegmentLayout, ratio: float, sample_ratio: float):
    ns = tuple(max(1, int(n * sample_ratio)) if n > 0 else 0 for n in layout.numels)
    ks = tuple(min(s, max(1, int(n * ratio * sample_ratio))) if n > 0 else 0 for n, s in zip(layout.numels, ns))
    return ns, ks


def dgc_capacity(layout: SegmentLayout, ratio: float, capacity: float) -> int:
    """Payload capacity: ``capacity`` x the summed per-segment targets max(1, ratio * n_i)
    (the refinement aims at [0.7, 1.3] x target; 2.0 leaves room for the segments that end the
    10 refinements outside that band), never more than the bucket."""
    tgt = sum(max(1.0, n * ratio) for n in layout.numels if n > 0)
    return max(1, min(layout.total, int(math.ceil(capacity * tgt))))


def dgc_select(x: torch.Tensor, layout: SegmentLayout, ratio: float, sample_ratio: float, max_iters: int,
               seed: int, cap: int, step: Optional[torch.Tensor] = None, vmask: Optional[torch.Tensor] = None,
               umask: Optional[torch.Tensor] = None, compensate: Optional[Tuple[float, bool]] = None
               ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """DGC selection of |x| >= thr_i per segment into a capacity payload (header, values, indices).
    ``step``: device step counter mixed into the sampling seed on the device (graph replays draw
    fresh samples); ``vmask`` / ``umask``: DgcMemory's v / u, zeroed at the SENT entries.
    ``compensate=(momentum, first)`` (native, with vmask / umask): ``x`` is the RAW gradient and
    DgcMemory's compensate (u = m u + g; v = v + u) is fused into the selection -- the samples
    read the compensated values on the fly and the first refinement pass writes u and v -- so the
    selection runs on v without a separate pass over the bucket."""
    from .cappayload import sparse_payload

    ns, ks = _sizes(layout, ratio, sample_ratio)
    dev = x.device
    hdr, v, i = sparse_payload(dev, cap)
    if _native.use_native(x):
        C = _native.lib()
        slay = layout.cached(dev, f"dgc_sample_layout:{sample_ratio}",
                             lambda: SegmentLayout(ns, tuple((s,) for s in ns)))
        t = layout.device_tables(dev)

        def build():
            return {
                "samp_off": torch.tensor(slay.offsets, dtype=torch.int64, device=dev),
                "target": torch.tensor([n * ratio for n in layout.numels], dtype=torch.float32, device=dev),
                "thr": torch.empty(layout.n_seg, dtype=torch.float32, device=dev),
                "count": torch.empty(32 * layout.n_seg, dtype=torch.int32, device=dev),  # tree counts + steps
                "done": torch.empty(layout.n_seg, dtype=torch.int32, device=dev),
                # per-chunk tree counts, final counted node per segment, chunk output offsets: the
                # compaction places every chunk at a scanned offset (no payload-counter atomics)
                "ccnt": torch.empty(32 * max(1, t["n_chunks"]), dtype=torch.int32, device=dev),
                "fnode": torch.empty(layout.n_seg, dtype=torch.int32, device=dev),
                "coff": torch.empty(max(1, t["n_chunks"]), dtype=torch.int32, device=dev),
                "samples": torch.empty(max(1, slay.total), dtype=torch.float32, device=dev),
            }

        ws = layout.cached(dev, f"dgc_ws:{ratio}:{sample_ratio}", build)
        sd = seed & 0xFFFFFFFFFFFFFFFF
        sd = sd - (1 << 64) if sd >= (1 << 63) else sd
        samples = ws["samples"][: slay.total]
        fuse = compensate is not None and vmask is not None and umask is not None
        cu, cv = (umask, vmask) if fuse else (None, None)
        mom, first = compensate if fuse else (0.0, False)
        C.dgc_sample(x, t["offsets"], ws["samp_off"], sd, step, samples, cu, cv, float(mom), bool(first))
        tw = _topk_ws(slay, ks, dev)
        # exact k'-th largest |sample| per segment + the refinement state, one launch
        C.dgc_select_init(samples, ws["samp_off"], tw["kseg"], tw["state"], ws["thr"], ws["count"], ws["done"],
                          ws["fnode"])
        C.dgc_refine(x, tw["state"], ws["target"], max_iters, ws["thr"], ws["count"], ws["done"], t["seg"],
                     t["begin"], t["end"], ws["ccnt"], ws["fnode"], cu, cv, float(mom), bool(first), init=False)
        sel = vmask if fuse else x  # after the fused refinement v holds the compensated values
        C.dgc_compact(sel, ws["thr"], v, i, hdr[:1], t["seg"], t["begin"], t["end"], ws["ccnt"], ws["fnode"],
                      ws["coff"], vmask, umask)
        return hdr, v, i
    if compensate is not None:
        raise ValueError("fused compensate needs the native path")
    # ---- PyTorch reference path (per segment, reference dgc.py:12-43 semantics)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    idxs = []
    for (si, o, n), s, k in zip(layout.segments(), ns, ks):
        if n == 0:
            continue
        seg = x[o:o + n]
        pos = (torch.rand(s, generator=gen, device=dev) * n).long().clamp_max(n - 1)
        thr = torch.topk(seg[pos].abs(), k).values.min()
        target = n * ratio
        mask = seg.abs() >= thr
        sel = mask.sum()
        for _ in range(max_iters):
            if sel > 1.3 * target:
                thr = 1.3 * thr
            elif sel < 0.7 * target:
                thr = 0.7 * thr
            else:
                break
            mask = seg.abs() >= thr
            sel = mask.sum()
        (ii,) = torch.where(mask)
        idxs.append(ii + o)
    cat_i = torch.cat(idxs) if idxs else torch.empty(0, dtype=torch.int64, device=dev)
    hdr.zero_()
    hdr[0] = cat_i.numel()
    hdr[1] = cap
    s_ = cat_i[:cap]
    v[: s_.numel()] = x[s_]
    i[: s_.numel()] = s_.to(torch.int32)
    for m in (vmask, umask):
        if m is not None:
            m[s_] = 0.0
    return hdr, v, i
