"""DGC threshold selection (native: csrc/kernels/dgc.hip + the segmented radix select)."""
from __future__ import annotations

from typing import Tuple

import torch

from . import _native
from .layout import SegmentLayout
from .topk import _workspace as _topk_ws


def _sizes(layout: SegmentLayout, ratio: float, sample_ratio: float):
    ns = tuple(max(1, int(n * sample_ratio)) if n > 0 else 0 for n in layout.numels)
    ks = tuple(min(s, max(1, int(n * ratio * sample_ratio))) if n > 0 else 0 for n, s in zip(layout.numels, ns))
    return ns, ks


def dgc_select(x: torch.Tensor, layout: SegmentLayout, ratio: float, sample_ratio: float, max_iters: int,
               seed: int) -> Tuple[torch.Tensor, torch.Tensor]:
    from ..parallel.comm import PayloadBuilder

    ns, ks = _sizes(layout, ratio, sample_ratio)
    dev = x.device
    if _native.use_native(x):
        C = _native.lib()
        slay = layout.cached(dev, f"dgc_sample_layout:{sample_ratio}",
                             lambda: SegmentLayout(ns, tuple((s,) for s in ns)))
        st = slay.device_tables(dev)
        t = layout.device_tables(dev)

        def build():
            return {
                "samp_off": torch.tensor(slay.offsets, dtype=torch.int64, device=dev),
                "target": torch.tensor([n * ratio for n in layout.numels], dtype=torch.float32, device=dev),
                "thr": torch.empty(layout.n_seg, dtype=torch.float32, device=dev),
                "count": torch.empty(layout.n_seg, dtype=torch.int32, device=dev),
                "done": torch.empty(layout.n_seg, dtype=torch.int32, device=dev),
                "samples": torch.empty(max(1, slay.total), dtype=torch.float32, device=dev),
                "cnt": torch.zeros(1, dtype=torch.int32, device=dev),
            }

        ws = layout.cached(dev, f"dgc_ws:{ratio}:{sample_ratio}", build)
        sd = seed & 0xFFFFFFFFFFFFFFFF
        sd = sd - (1 << 64) if sd >= (1 << 63) else sd
        samples = ws["samples"][: slay.total]
        C.dgc_sample(x, t["offsets"], ws["samp_off"], sd, samples)
        tw = _topk_ws(slay, ks, dev)
        C.topk_select(samples, None, samples, 1.0, 1.0, 0, st["seg"], st["begin"], st["end"], tw["kseg"],
                      tw["state"], tw["hist"])
        C.dgc_refine(x, tw["state"], ws["target"], max_iters, ws["thr"], ws["count"], ws["done"], t["seg"],
                     t["begin"], t["end"])
        cap_v = torch.empty(x.numel(), dtype=torch.float32, device=dev)
        cap_i = torch.empty(x.numel(), dtype=torch.int32, device=dev)
        C.dgc_compact(x, ws["thr"], cap_v, cap_i, ws["cnt"], t["seg"], t["begin"], t["end"])
        s = int(ws["cnt"].item())
        v, i = PayloadBuilder(dev, [(torch.float32, (s,)), (torch.int32, (s,))]).tensors
        if s:
            v.copy_(cap_v[:s])
            i.copy_(cap_i[:s])
        return v, i
    # ---- PyTorch reference path (per segment, reference dgc.py:12-43 semantics)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    vals, idxs = [], []
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
        vals.append(seg[ii])
        idxs.append((ii + o).to(torch.int32))
    cat_v = torch.cat(vals) if vals else torch.empty(0, device=dev)
    cat_i = torch.cat(idxs) if idxs else torch.empty(0, dtype=torch.int32, device=dev)
    v, i = PayloadBuilder(dev, [(torch.float32, (cat_v.numel(),)), (torch.int32, (cat_i.numel(),))]).tensors
    v.copy_(cat_v)
    i.copy_(cat_i)
    return v, i
