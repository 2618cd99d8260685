"""Quantizer ops: QSGD, TernGrad, Natural, 8-bit table (native: csrc/kernels/quant.hip).

The PyTorch paths are the CPU oracles (same math, torch RNG instead of Philox).
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native
from .layout import SegmentLayout
from .segstats import expand

U8_TABLE = torch.tensor([
    1.5000001e-06, 2.7500000e-06, 7.2499997e-06, 1.8750001e-05, 3.6250000e-05, 5.8749996e-05, 8.6249995e-05,
    1.4375000e-04, 2.3125000e-04, 3.1875001e-04, 4.0625001e-04, 5.1874999e-04, 6.5624999e-04, 7.9374999e-04,
    9.3124999e-04, 1.2187500e-03, 1.6562500e-03, 2.0937501e-03, 2.5312500e-03, 2.9687500e-03, 3.4062499e-03,
    3.8437501e-03, 4.2812498e-03, 4.8437500e-03, 5.5312500e-03, 6.2187500e-03, 6.9062500e-03, 7.5937500e-03,
    8.2812496e-03, 8.9687500e-03, 9.6562495e-03, 1.1093750e-02, 1.3281250e-02, 1.5468750e-02, 1.7656250e-02,
    1.9843750e-02, 2.2031249e-02, 2.4218749e-02, 2.6406251e-02, 2.8593751e-02, 3.0781250e-02, 3.2968748e-02,
    3.5156250e-02, 3.7343752e-02, 3.9531250e-02, 4.1718751e-02, 4.3906249e-02, 4.6718750e-02, 5.0156251e-02,
    5.3593751e-02, 5.7031251e-02, 6.0468748e-02, 6.3906237e-02, 6.7343749e-02, 7.0781253e-02, 7.4218743e-02,
    7.7656247e-02, 8.1093743e-02, 8.4531240e-02, 8.7968737e-02, 9.1406241e-02, 9.4843738e-02, 9.8281242e-02,
    1.0546875e-01, 1.1640625e-01, 1.2734374e-01, 1.3828126e-01, 1.4921875e-01, 1.6015625e-01, 1.7109375e-01,
    1.8203124e-01, 1.9296876e-01, 2.0390625e-01, 2.1484375e-01, 2.2578125e-01, 2.3671874e-01, 2.4765626e-01,
    2.5859374e-01, 2.6953125e-01, 2.8046876e-01, 2.9140624e-01, 3.0234376e-01, 3.1328124e-01, 3.2421875e-01,
    3.3515626e-01, 3.4609374e-01, 3.5703126e-01, 3.6796874e-01, 3.7890625e-01, 3.8984376e-01, 4.0078124e-01,
    4.1171876e-01, 4.2265624e-01, 4.3359375e-01, 4.4453126e-01, 4.5859376e-01, 4.7578123e-01, 4.9296874e-01,
    5.1015621e-01, 5.2734375e-01, 5.4453123e-01, 5.6171870e-01, 5.7890624e-01, 5.9609371e-01, 6.1328125e-01,
    6.3046873e-01, 6.4765620e-01, 6.6484374e-01, 6.8203121e-01, 6.9921869e-01, 7.1640623e-01, 7.3359370e-01,
    7.5078118e-01, 7.6796871e-01, 7.8515619e-01, 8.0234367e-01, 8.1953120e-01, 8.3671868e-01, 8.5390615e-01,
    8.7109369e-01, 8.8828117e-01, 9.0546864e-01, 9.2265618e-01, 9.3984365e-01, 9.5703113e-01, 9.7421867e-01,
    9.9140614e-01, 9.9570298e-01], dtype=torch.float32)


def _gen(seed: int, device) -> torch.Generator:
    g = torch.Generator(device=device)
    g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    return g


def _tables(layout, device):
    return layout.device_tables(device)


def _seed64(seed: int) -> int:
    seed &= 0xFFFFFFFFFFFFFFFF
    return seed - (1 << 64) if seed >= (1 << 63) else seed


# ------------------------------------------------------------------------------ QSGD
def qsgd_quantize(x: torch.Tensor, layout: SegmentLayout, norms: torch.Tensor, s: int, seed: int,
                  codes: torch.Tensor, resid: Optional[torch.Tensor] = None,
                  step: Optional[torch.Tensor] = None) -> None:
    """``step``: optional device int64 counter mixed into ``seed`` by the kernel (graph replay)."""
    if _native.use_native(x):
        t = _tables(layout, x.device)
        _native.lib().qsgd_quantize(x, norms, float(s), _seed64(seed), step, codes, resid, t["seg"], t["begin"], t["end"])
        return
    nrm = expand(norms, layout)
    inv = torch.where(nrm > 0, s / nrm, torch.zeros_like(nrm))
    lvl = inv * x.abs()
    fl = lvl.floor()
    u = torch.rand(x.shape, generator=_gen(seed, x.device), device=x.device)
    q = fl + (u < (lvl - fl)).float()
    code = torch.sign(x) * q
    codes.copy_(code.to(codes.dtype))
    if resid is not None:
        resid.copy_(x - nrm / s * code)


def qsgd_pack_bits(s: int) -> int:
    """Bits per bit-packed code (ceil(log2(2s+1)), rounded to 2 or 4 so codes never
    straddle a byte): 2 for s = 1, 4 for s <= 7, 0 = no packing (int8 / wider codes)."""
    return 2 if s == 1 else (4 if 1 < s <= 7 else 0)


def qsgd_pack(codes: torch.Tensor, s: int, bits: int, out: torch.Tensor) -> None:
    """int8 codes in [-s, s] -> ``bits``-bit fields (code + s), element i at bit i*bits of ``out``."""
    if _native.use_native(codes):
        _native.lib().qsgd_pack(codes, int(s), int(bits), out)
        return
    n = codes.numel()
    per = 8 // bits
    v = (codes.to(torch.int32) + s)
    pad = (-n) % per
    if pad:
        v = torch.cat([v, torch.zeros(pad, dtype=torch.int32, device=v.device)])
    v = v.view(-1, per)
    shifts = torch.arange(per, device=v.device, dtype=torch.int32) * bits
    packed = (v << shifts).sum(1).to(torch.uint8)
    out[:packed.numel()].copy_(packed)


def _unpack(row: torch.Tensor, n: int, s: int, bits: int) -> torch.Tensor:
    per = 8 // bits
    b = row[: (n * bits + 7) // 8].to(torch.int32)
    shifts = torch.arange(per, device=row.device, dtype=torch.int32) * bits
    v = ((b.unsqueeze(1) >> shifts) & ((1 << bits) - 1)).reshape(-1)[:n]
    return (v - s).float()


def qsgd_aggregate(base, rank_stride, codes_off, norms_off, code_dtype, n_ranks, s, layout, out, scale,
                   accumulate=False, shared_norms=None, packed_bits: int = 0):
    """Decode-sum of W payload rows.  ``shared_norms``: the shared-scale variant's all-reduced
    norms, used for every row (the rows then carry codes only; ``norms_off`` is ignored).
    ``packed_bits`` (2 / 4): the rows carry bit-packed codes (``qsgd_pack``)."""
    if _native.use_native(out):
        t = _tables(layout, out.device)
        if packed_bits:
            C = _native.lib()
            esz = C.QSGD_PACKED2 if packed_bits == 2 else C.QSGD_PACKED4
        else:
            esz = 3 if code_dtype == torch.float16 else torch.empty((), dtype=code_dtype).element_size()
        _native.lib().qsgd_aggregate(base, rank_stride, codes_off, norms_off, esz, n_ranks, float(s), scale, out,
                                     accumulate, t["seg"], t["begin"], t["end"], layout.n_seg, shared_norms)
        return
    esz = torch.empty((), dtype=code_dtype).element_size()
    acc = torch.zeros(layout.total, dtype=torch.float32, device=out.device)
    for r in range(n_ranks):
        row = base[r * rank_stride:]
        if packed_bits:
            q = _unpack(row[codes_off:], layout.total, s, packed_bits)
        else:
            q = row[codes_off:codes_off + esz * layout.total].view(code_dtype).float()
        nrm = shared_norms if shared_norms is not None else row[norms_off:norms_off + 4 * layout.n_seg].view(torch.float32)
        acc += expand(nrm, layout) / s * q
    acc *= scale
    if accumulate:
        out += acc
    else:
        out.copy_(acc)


# ------------------------------------------------------------------------------ TernGrad
def tern_quantize(x, layout, clips, scal, seed, words, resid=None, step=None):
    if _native.use_native(x):
        t = _tables(layout, x.device)
        _native.lib().tern_quantize(x, clips, scal, _seed64(seed), step, words, resid, t["seg"], t["begin"], t["end"],
                                    t["offsets"], t["word_off"], layout.n_words)
        return
    from .signbits import pack_bits_torch

    c = expand(clips, layout)
    sc = expand(scal, layout)
    gcl = torch.maximum(torch.minimum(x, c), -c)
    u = torch.rand(x.shape, generator=_gen(seed, x.device), device=x.device) * sc
    t = torch.where(u < gcl.abs(), torch.sign(gcl), torch.zeros_like(gcl))
    nz = pack_bits_torch(t != 0, layout)
    ng = pack_bits_torch(t < 0, layout)
    words.view(-1, 2)[:, 0] = nz
    words.view(-1, 2)[:, 1] = ng
    if resid is not None:
        resid.copy_(x - t * sc)


def tern_aggregate(base, rank_stride, words_off, scal_off, n_ranks, layout, out, scale, accumulate=False):
    if _native.use_native(out):
        t = _tables(layout, out.device)
        _native.lib().tern_aggregate(base, rank_stride, words_off, scal_off, n_ranks, scale, out, accumulate,
                                     t["seg"], t["begin"], t["end"], t["offsets"], t["word_off"], layout.n_words)
        return
    from .signbits import unpack_bits_torch

    nw = layout.n_words
    acc = torch.zeros(layout.total, dtype=torch.float32, device=out.device)
    for r in range(n_ranks):
        row = base[r * rank_stride:]
        w = row[words_off:words_off + 16 * nw].view(torch.int64).view(-1, 2)
        nz = unpack_bits_torch(w[:, 0].contiguous(), layout)
        ng = unpack_bits_torch(w[:, 1].contiguous(), layout)
        sc = expand(row[scal_off:scal_off + 4 * layout.n_seg].view(torch.float32), layout)
        acc += torch.where(nz, torch.where(ng, -sc, sc), torch.zeros_like(sc))
    acc *= scale
    if accumulate:
        out += acc
    else:
        out.copy_(acc)


# ------------------------------------------------------------------------------ Natural
def natural_encode(x, seed, codes, resid=None, step=None):
    if _native.use_native(x):
        _native.lib().natural_encode(x, _seed64(seed), step, codes, resid)
        return
    bits = x.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    sign = bits & 0x80000000
    expo = bits & 0x7F800000
    mant = bits & 0x007FFFFF
    rnd = torch.randint(0, 1 << 23, x.shape, generator=_gen(seed, x.device), device=x.device)
    expo = torch.where(mant > rnd, expo + 0x00800000, expo)
    expo = expo.clamp(0x09000000, 0x48800000)
    code = (sign >> 24) | ((expo >> 23) - 18)
    codes.copy_(code.to(torch.uint8))
    if resid is not None:
        resid.copy_(x - natural_decode_torch(codes))


def natural_decode_torch(codes: torch.Tensor) -> torch.Tensor:
    c = codes.to(torch.int32)
    e = c & 0x7F
    f = ((e + 18) << 23).view(torch.float32)
    f = torch.where(c > 127, -f, f)
    return torch.where(e >= 1, f, torch.zeros_like(f))


def natural_aggregate(base, rank_stride, n_ranks, out, scale, accumulate=False):
    if _native.use_native(out):
        _native.lib().natural_aggregate(base, rank_stride, n_ranks, scale, out, accumulate)
        return
    n = out.numel()
    acc = torch.zeros(n, dtype=torch.float32, device=out.device)
    for r in range(n_ranks):
        acc += natural_decode_torch(base[r * rank_stride:r * rank_stride + n])
    acc *= scale
    if accumulate:
        out += acc
    else:
        out.copy_(acc)


# ------------------------------------------------------------------------------ U8bit
def u8_bins_torch(v: torch.Tensor) -> torch.Tensor:
    tab = U8_TABLE.to(v.device)
    b = torch.searchsorted(tab, v.contiguous(), right=True) - 1
    return b.clamp(0, 126)


def u8_encode(x, layout, scales, codes, resid=None):
    if _native.use_native(x):
        t = _tables(layout, x.device)
        _native.lib().u8_encode(x, scales, codes, resid, t["seg"], t["begin"], t["end"])
        return
    sc = expand(scales, layout)
    inv = torch.where(sc > 0, 1.0 / sc, torch.zeros_like(sc))
    b = u8_bins_torch(x.abs() * inv)
    code = torch.sign(x).long() * b
    codes.copy_(code.to(torch.int8))
    if resid is not None:
        resid.copy_(x - u8_decode_torch(codes, sc))


def u8_decode_torch(codes, sc_expanded):
    q = codes.long()
    tab = U8_TABLE.to(codes.device)
    return torch.sign(q).float() * tab[q.abs()] * sc_expanded


def u8_aggregate(base, rank_stride, codes_off, scal_off, n_ranks, layout, out, scale, accumulate=False):
    if _native.use_native(out):
        t = _tables(layout, out.device)
        _native.lib().u8_aggregate(base, rank_stride, codes_off, scal_off, n_ranks, scale, out, accumulate,
                                   t["seg"], t["begin"], t["end"], layout.n_seg)
        return
    acc = torch.zeros(layout.total, dtype=torch.float32, device=out.device)
    for r in range(n_ranks):
        row = base[r * rank_stride:]
        q = row[codes_off:codes_off + layout.total].view(torch.int8)
        sc = expand(row[scal_off:scal_off + 4 * layout.n_seg].view(torch.float32), layout)
        acc += u8_decode_torch(q, sc)
    acc *= scale
    if accumulate:
        out += acc
    else:
        out.copy_(acc)
