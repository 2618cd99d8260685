"""Random-K index generation + gather/scatter (native: csrc/kernels/sparsify.hip).

Index j of segment s is ``seg_off[s] + pi_{seed_s}(j)`` where pi is the keyed Feistel
permutation of csrc/include/grace_rand.h.  The PyTorch implementation below uses the SAME
32-bit integer arithmetic, so CPU and GPU select identical indices for the same seed.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch

from . import _native
from .layout import SegmentLayout

M32 = 0xFFFFFFFF
GOLDEN = 0x9E3779B9


def fnv1a64(data: bytes) -> int:
    h = 0xCBF29CE484222325
    for b in data:
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _fmix32_int(h: int) -> int:
    h &= M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


def _fmix32_t(h: torch.Tensor) -> torch.Tensor:
    h = h & M32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & M32
    h = h ^ (h >> 16)
    return h


def feistel_key(seed: int, n: int):
    bits = 2
    while bits < 64 and (1 << bits) < n:
        bits += 1
    if bits & 1:
        bits += 1
    half = bits >> 1
    mask = M32 if half >= 32 else (1 << half) - 1
    lo, hi = seed & M32, (seed >> 32) & M32
    ks = [_fmix32_int(lo ^ ((GOLDEN * (i + 1)) & M32) ^ _fmix32_int((hi + i) & M32)) for i in range(4)]
    return ks, half, mask


def _round4(x: torch.Tensor, ks, half, mask) -> torch.Tensor:
    L = (x >> half) & mask
    R = x & mask
    for k in ks:
        f = _fmix32_t(R ^ k) & mask
        L, R = R, L ^ f
    return (L << half) | R


def feistel_perm(j: torch.Tensor, n: int, seed: int) -> torch.Tensor:
    """pi_seed(j) for an int64 tensor j of values < n (cycle walking)."""
    ks, half, mask = feistel_key(seed, n)
    y = _round4(j, ks, half, mask)
    bad = y >= n
    while bool(bad.any()):
        y = torch.where(bad, _round4(y, ks, half, mask), y)
        bad = y >= n
    return y


_GOLDEN = 0x9E3779B97F4A7C15


def mix_step(seed: int, step: int) -> int:
    """seed ^ step * golden (mod 2^64): host twin of the kernels' device-step mixing."""
    return (seed ^ (step * _GOLDEN)) & 0xFFFFFFFFFFFFFFFF


def indices(layout: SegmentLayout, ks: Sequence[int], seeds: Sequence[int], device="cpu",
            step: int = 0) -> torch.Tensor:
    out = []
    for (i, o, n), k, sd in zip(layout.segments(), ks, seeds):
        if k:
            out.append(feistel_perm(torch.arange(k, dtype=torch.int64, device=device), n, mix_step(sd, step)) + o)
    return torch.cat(out) if out else torch.empty(0, dtype=torch.int64, device=device)


def _tables(layout: SegmentLayout, ks: Sequence[int], seeds: Sequence[int], device, step: int, step_t):
    """Device tables; with a device step counter the seed table is step-independent and
    cached (no per-step host->device copy: capturable in a HIP graph)."""
    def build():
        off = [0]
        for k in ks:
            off.append(off[-1] + k)
        return {
            "seg_off": torch.tensor(layout.offsets, dtype=torch.int64, device=device),
            "out_off": torch.tensor(off, dtype=torch.int64, device=device),
        }

    def seed_tensor(ss):
        return torch.tensor([s - (1 << 64) if s >= (1 << 63) else s for s in ss], dtype=torch.int64)

    t = layout.cached(device, f"randk:{hash(tuple(ks))}", build)
    if step_t is not None:
        sd = layout.cached(device, f"randk_seeds:{hash(tuple(seeds))}", lambda: seed_tensor(seeds).to(device))
        return t, sd
    sd = seed_tensor([mix_step(s, step) for s in seeds])
    return t, sd.to(device, non_blocking=True)


def gather(x: torch.Tensor, layout, ks, seeds, zero_selected: bool = False, step: int = 0,
           step_t: Optional[torch.Tensor] = None) -> torch.Tensor:
    """vals[j] = x[idx_j]; optionally x[idx_j] = 0 afterwards (residual update).

    Effective seed of segment s: ``seeds[s] ^ step * golden`` with the step taken from the
    device counter ``step_t`` when given (native path), else from the host ``step``."""
    K = sum(ks)
    vals = torch.empty(K, dtype=torch.float32, device=x.device)
    if _native.use_native(x):
        t, sd = _tables(layout, ks, seeds, x.device, step, step_t)
        _native.lib().randk_gather(x, t["seg_off"], t["out_off"], sd, step_t, vals, x if zero_selected else None)
        return vals
    idx = indices(layout, ks, seeds, x.device, step)
    vals.copy_(x[idx])
    if zero_selected:
        x[idx] = 0.0
    return vals


def scatter(vals_rows: torch.Tensor, layout, ks, seeds, out: torch.Tensor, scale: float,
            accumulate: bool = False, step: int = 0, step_t: Optional[torch.Tensor] = None) -> None:
    """out[idx_j] (+)= scale * sum_r vals_rows[r, j] (rank-ordered sum)."""
    K = sum(ks)
    if vals_rows.dim() == 1:
        vals_rows = vals_rows.view(1, -1)
    if _native.use_native(out):
        t, sd = _tables(layout, ks, seeds, out.device, step, step_t)
        stride = vals_rows.stride(0) if vals_rows.size(0) > 1 else K
        assert vals_rows.stride(1) == 1
        _native.lib().randk_scatter(vals_rows, stride, vals_rows.size(0), K, t["seg_off"], t["out_off"], sd, step_t,
                                    out, scale, accumulate)
        return
    idx = indices(layout, ks, seeds, out.device, step)
    acc = vals_rows[0, :K].clone()
    for r in range(1, vals_rows.size(0)):
        acc += vals_rows[r, :K]
    acc *= scale
    if accumulate:
        out.index_add_(0, idx, acc)
    else:
        out[idx] = acc
