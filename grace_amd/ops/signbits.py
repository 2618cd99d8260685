"""1-bit sign packing / majority vote / weighted decode (native: csrc/kernels/signbits.hip).

Bit layout: segment s owns uint64 words [word_off[s], word_off[s+1]); bit l of word g is
element 64*g + l of the segment (what a wave64 ``__ballot`` produces).  Words travel as int64.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native
from .layout import SegmentLayout

_SHIFTS = {}


def _shifts(device):
    t = _SHIFTS.get(device)
    if t is None:
        t = _SHIFTS[device] = torch.arange(64, dtype=torch.int64, device=device)
    return t


def pack_bits_torch(bits: torch.Tensor, layout: SegmentLayout) -> torch.Tensor:
    """bool[n_total] -> int64 words (per-segment 64-element groups)."""
    out = []
    sh = _shifts(bits.device)
    for i, o, n in layout.segments():
        ng = (n + 63) // 64
        b = torch.zeros(ng * 64, dtype=torch.int64, device=bits.device)
        b[:n] = bits[o:o + n].to(torch.int64)
        out.append((b.view(ng, 64) << sh).sum(dim=1))
    return torch.cat(out) if out else torch.empty(0, dtype=torch.int64, device=bits.device)


def unpack_bits_torch(words: torch.Tensor, layout: SegmentLayout) -> torch.Tensor:
    """int64 words -> bool[n_total]."""
    out = []
    sh = _shifts(words.device)
    wo = layout.word_offsets()
    for i, o, n in layout.segments():
        w = words[wo[i]:wo[i + 1]]
        out.append((((w.unsqueeze(1) >> sh) & 1).view(-1)[:n]).bool())
    return torch.cat(out) if out else torch.empty(0, dtype=torch.bool, device=words.device)


def sign_pack(g: torch.Tensor, layout: SegmentLayout, words: torch.Tensor, *, neg: bool = False,
              r: Optional[torch.Tensor] = None, r_valid: bool = False, beta: float = 1.0, gamma: float = 1.0,
              mom: Optional[torch.Tensor] = None, mom_beta: float = 0.0, mom_valid: bool = False,
              vT: Optional[torch.Tensor] = None, vF: Optional[torch.Tensor] = None,
              resid: Optional[torch.Tensor] = None) -> None:
    """words <- bits of (x >= 0) [or x < 0 when ``neg``] where x is the (compensated) gradient,
    optionally through Signum momentum; optional residual r' = x - (bit ? vT : vF) per segment."""
    ef = 1 if (r is not None and r_valid) else 0
    if _native.use_native(g):
        t = layout.device_tables(g.device)
        _native.lib().sign_pack(g, r if ef else None, ef, beta, gamma, mom, mom_beta, mom_valid, vT, vF, resid, neg,
                                words, t["seg"], t["begin"], t["end"], t["offsets"], t["word_off"], layout.n_words)
        return
    x = beta * r + gamma * g if ef else g
    v = x
    if mom is not None:
        v = (1.0 - mom_beta) * x + mom_beta * mom if mom_valid else x.clone()
        mom.copy_(v)
    bits = (v < 0) if neg else (v >= 0)
    words.copy_(pack_bits_torch(bits, layout))
    if resid is not None:
        from .segstats import expand

        dec = torch.where(bits, expand(vT, layout), expand(vF, layout))
        resid.copy_(x - dec)


def sign_unpack(base: torch.Tensor, rank_stride: int, words_off: int, vals_off: int, n_ranks: int, layout,
                out: torch.Tensor, *, vote: bool, scale: float = 1.0, accumulate: bool = False) -> None:
    """VOTE: out = +1 if 2*#(bit=1) >= W else -1.  VALUE: out = scale * sum_r (bit ? vT_r : vF_r)
    with per-rank [vT_0, vF_0, vT_1, vF_1, ...] fp32 at ``vals_off``."""
    if _native.use_native(out):
        t = layout.device_tables(out.device)
        _native.lib().sign_unpack(base, rank_stride, words_off, vals_off, n_ranks, vote, scale, out, accumulate,
                                  t["seg"], t["begin"], t["end"], t["offsets"], t["word_off"], layout.n_words)
        return
    nw = layout.n_words
    acc = torch.zeros(layout.total, dtype=torch.float32, device=out.device)
    ones = torch.zeros(layout.total, dtype=torch.int32, device=out.device)
    from .segstats import expand

    for rk in range(n_ranks):
        row = base[rk * rank_stride:]
        words = row[words_off:words_off + 8 * nw].view(torch.int64)
        bits = unpack_bits_torch(words, layout)
        if vote:
            ones += bits.int()
        else:
            vals = row[vals_off:vals_off + 8 * layout.n_seg].view(torch.float32).view(-1, 2)
            acc += torch.where(bits, expand(vals[:, 0].contiguous(), layout), expand(vals[:, 1].contiguous(), layout))
    res = torch.where(2 * ones >= n_ranks, 1.0, -1.0) if vote else acc * scale
    if accumulate:
        out += res
    else:
        out.copy_(res)
