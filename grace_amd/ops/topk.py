"""Segmented exact Top-K with fused error feedback (native: ``csrc/kernels/topk.hip``).

Reference: /root/reference/grace_dl/dist/compressor/topk.py:6-36 (per-tensor
``torch.topk(|x|, k)`` + gather + scatter decompress) and
/root/reference/grace_dl/dist/memory/residual.py:10-20 (compensate / update).

Payload format (one collective per bucket instead of two per tensor): one 16-B aligned
buffer holding [ fp32 values (K) | int32 flat indices (K) ].
The TF backend's layout (fp32 values + int32 indices in one tensor,
/root/reference/grace_dl/tensorflow/compressor/topk.py:32-35) - 8 bytes per element instead
of the dist backend's 12.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch

from . import _native
from .layout import SegmentLayout


def k_per_segment(layout: SegmentLayout, ratio: float) -> Tuple[int, ...]:
    """k_i = max(1, int(n_i * ratio)) -- reference topk.py:7 (cached per layout)."""
    return layout.cached("host", f"k:{ratio!r}",
                         lambda: tuple(min(n, max(1, int(n * ratio))) if n > 0 else 0 for n in layout.numels))


def _workspace(layout: SegmentLayout, ks: Sequence[int], device):
    def build():
        n = layout.n_seg
        off = [0]
        for k in ks:
            off.append(off[-1] + k)
        return {
            "kseg": torch.tensor(list(ks), dtype=torch.int32, device=device),
            "out_off": torch.tensor(off, dtype=torch.int64, device=device),
            "K": off[-1],
            "state": torch.zeros(2 * n, dtype=torch.int32, device=device),
            "hist": torch.zeros(n * 2048, dtype=torch.int32, device=device),
            "counters": torch.zeros(2 * n, dtype=torch.int32, device=device),
        }

    return layout.cached(device, f"topk_ws:{hash(tuple(ks))}", build)


TOPK_CHUNK = 16384  # elements per workgroup in the two streaming passes


def _two_pass_ws(layout: SegmentLayout, device):
    """Device state of the two-pass pipeline (csrc/kernels/topk.hip ``topk_ef_bucket``): candidate
    buffers (value + index, one slice per chunk, sized like the bucket so any distribution fits),
    per-chunk take/candidate/above-prefix counts and the 3 per-segment counters."""
    def build():
        n_chunks = layout.device_tables(device, TOPK_CHUNK)["n_chunks"]
        i32 = dict(dtype=torch.int32, device=device)
        return {
            "ctr": torch.zeros(3 * layout.n_seg, **i32),
            "ccnt": torch.zeros(3 * max(1, n_chunks), **i32),
            "cand_val": torch.empty(max(1, layout.total), dtype=torch.float32, device=device),
            "cand_idx": torch.empty(max(1, layout.total), **i32),
        }

    return layout.cached(device, "topk2_ws", build)


def topk_ef(
    g: torch.Tensor,
    layout: SegmentLayout,
    ks: Sequence[int],
    resid: Optional[torch.Tensor] = None,
    resid_valid: bool = False,
    beta: float = 1.0,
    gamma: float = 1.0,
    out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
    key: Optional[str] = None,
) -> Tuple[torch.Tensor, torch.Tensor]:
    """Compensate + select + (residual update) over a flat bucket.

    ``g``      flat fp32 gradient bucket (read only)
    ``resid``  flat fp32 residual buffer or None (NoneMemory). If given it is read (when
               ``resid_valid``), overwritten with x = beta*r + gamma*g and finally left holding
               x - decompress(compress(x)), i.e. x with the selected entries zeroed.
    returns (vals fp32[K], idx int32[K]) -- views of ONE buffer laid out as the packed wire
    format (grace_amd.parallel.comm.pack is then zero-copy).
    """
    assert g.dtype == torch.float32 and g.dim() == 1 and g.is_contiguous()
    K = sum(ks)
    if out is None:
        from ..parallel.comm import PayloadBuilder

        vals, idx = PayloadBuilder(g.device, [(torch.float32, (K,)), (torch.int32, (K,))], key=key).tensors
    else:
        vals, idx = out
    if _native.use_native(g):
        C = _native.lib()
        ws = _workspace(layout, ks, g.device)
        w2 = _two_pass_ws(layout, g.device)
        t = layout.device_tables(g.device, TOPK_CHUNK)
        x = resid if resid is not None else g
        mode = 1 if (resid is not None and resid_valid) else 0
        C.topk_ef(g, x, beta, gamma, mode, resid is not None, t["seg"], t["begin"], t["end"],
                  t["seg_chunk_begin"], ws["kseg"], ws["state"], ws["hist"], w2["ctr"], w2["ccnt"],
                  ws["out_off"], vals, idx, w2["cand_val"], w2["cand_idx"])
        return vals, idx
    # ---- PyTorch reference path (CPU / oracle)
    if resid is not None:
        if resid_valid:
            x = beta * resid + gamma * g
        else:
            x = g.clone()
        resid.copy_(x)
        x = resid
    else:
        x = g
    p = 0
    for (i, o, n), k in zip(layout.segments(), ks):
        if k == 0:
            continue
        seg = x[o:o + n]
        _, li = torch.topk(seg.abs(), k, sorted=False)
        vals[p:p + k] = seg[li]
        idx[p:p + k] = (li + o).to(torch.int32)
        if resid is not None:
            seg[li] = 0.0
        p += k
    return vals, idx


def scatter_add(vals: torch.Tensor, idx: torch.Tensor, out: torch.Tensor, scale: float = 1.0,
                accumulate: bool = True) -> None:
    """out[idx] (+)= vals * scale for one rank's payload (indices unique within a payload)."""
    if _native.use_native(out):
        _native.lib().sparse_scatter_add(vals, idx, out, scale, accumulate)
        return
    il = idx.long()
    if accumulate:
        out.index_add_(0, il, vals * scale)
    else:
        out[il] = vals * scale
