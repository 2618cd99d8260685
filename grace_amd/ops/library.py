"""Device kernels of the ``grace`` dispatcher operators (schemas + Meta kernels:
csrc/ops_library.cpp ``TORCH_LIBRARY(grace, m)``).

Each op is the per-tensor GRACE contract of one reference compressor:

=============================  =====================================================================
``grace::topk_compress``       /root/reference/grace_dl/dist/compressor/topk.py:6-30 +
                               memory/residual.py:10-20 (fused error feedback)
``grace::sparse_decompress``   topk.py:14-18 / allgather.py:40-45 (scatter of every rank's payload)
``grace::randomk_*``           compressor/randomk.py:6-40 (shared indices; here a keyed Feistel
                               permutation instead of a reseeded global RNG)
``grace::sign_*``              compressor/signsgd.py:11-30 (1 bit / element, majority vote)
``grace::qsgd_*``              compressor/qsgd.py:12-38 (int8 below 128 levels, int16 above)
``grace::natural_*``           compressor/natural.py:13-40
=============================  =====================================================================

The CUDA (HIP) registrations run the same native gfx950 launchers as the bucketed engine (a
one-segment layout); the CPU registrations run the PyTorch reference path of those helpers.  The
stochastic ops take an explicit ``seed`` (reproducible, rank-independent where the reference
needs it: Random-K).  Registered on import of :mod:`grace_amd.ops` (the schemas come with the
native library; without it they are defined here with Python fake kernels instead).
"""
from __future__ import annotations

from typing import List

import torch

from . import _native
from .layout import layout_for

_LIB = None
_SCHEMAS = {
    "topk_compress": "topk_compress(Tensor grad, Tensor? residual, float ratio, float beta=1.0, float gamma=1.0)"
                     " -> (Tensor values, Tensor indices, Tensor residual_out)",
    "sparse_decompress": "sparse_decompress(Tensor values, Tensor indices, int[] shape, float scale=1.0) -> Tensor",
    "randomk_compress": "randomk_compress(Tensor grad, float ratio, int seed) -> Tensor",
    "randomk_decompress": "randomk_decompress(Tensor values, int[] shape, float ratio, int seed, float scale=1.0)"
                          " -> Tensor",
    "sign_compress": "sign_compress(Tensor grad) -> Tensor",
    "sign_decompress": "sign_decompress(Tensor words, int[] shape) -> Tensor",
    "qsgd_compress": "qsgd_compress(Tensor grad, int levels, int seed) -> (Tensor codes, Tensor norm)",
    "qsgd_decompress": "qsgd_decompress(Tensor codes, Tensor norms, int levels, int[] shape) -> Tensor",
    "natural_compress": "natural_compress(Tensor grad, int seed) -> Tensor",
    "natural_decompress": "natural_decompress(Tensor codes, int[] shape) -> Tensor",
}


def k_of(n: int, ratio: float) -> int:
    return min(n, max(1, int(n * ratio))) if n > 0 else 0


def _flat(t: torch.Tensor) -> torch.Tensor:
    """fp32, contiguous, 1-D, 16-B aligned (the native launchers' contract)."""
    f = t.reshape(-1)
    if f.dtype != torch.float32:
        f = f.float()
    if not f.is_contiguous() or f.data_ptr() % 16:
        f = f.contiguous().clone() if f.data_ptr() % 16 else f.contiguous()
    return f


def _numel(shape) -> int:
    n = 1
    for d in shape:
        n *= int(d)
    return n


# ------------------------------------------------------------------------------ Top-K
def topk_compress(grad, residual, ratio, beta=1.0, gamma=1.0):
    from .topk import k_per_segment, topk_ef

    g = _flat(grad)
    lay = layout_for([(g.numel(),)])
    ks = k_per_segment(lay, float(ratio))
    res = torch.empty_like(g)
    if residual is not None:
        res.copy_(residual.reshape(-1))
    vals = torch.empty(ks[0], dtype=torch.float32, device=g.device)
    idx = torch.empty(ks[0], dtype=torch.int32, device=g.device)
    topk_ef(g, lay, ks, resid=res, resid_valid=residual is not None, beta=float(beta), gamma=float(gamma),
            out=(vals, idx))
    return vals, idx, res.view(grad.shape)


def sparse_decompress(values, indices, shape, scale=1.0):
    """values / indices: [k] (one payload) or [W, k] (one row per rank, decoded in rank order)."""
    from .topk import scatter_add

    out = torch.zeros(_numel(shape), dtype=torch.float32, device=values.device)
    v = values.reshape(-1, values.shape[-1]) if values.dim() > 1 else values.reshape(1, -1)
    i = indices.reshape(v.shape).to(torch.int32)
    for r in range(v.shape[0]):  # indices are unique within one payload, not across ranks
        scatter_add(v[r].contiguous(), i[r].contiguous(), out, float(scale), accumulate=True)
    return out.view(list(shape))


# ------------------------------------------------------------------------------ Random-K
def randomk_compress(grad, ratio, seed):
    from . import randomk as RK

    g = _flat(grad)
    lay = layout_for([(g.numel(),)])
    ks = (k_of(g.numel(), float(ratio)),)
    return RK.gather(g, lay, ks, (int(seed) & 0xFFFFFFFFFFFFFFFF,))


def randomk_decompress(values, shape, ratio, seed, scale=1.0):
    from . import randomk as RK

    n = _numel(shape)
    lay = layout_for([(n,)])
    ks = (k_of(n, float(ratio)),)
    rows = values.reshape(-1, ks[0]).float().contiguous()
    out = torch.zeros(n, dtype=torch.float32, device=values.device)
    RK.scatter(rows, lay, ks, (int(seed) & 0xFFFFFFFFFFFFFFFF,), out, float(scale), accumulate=False)
    return out.view(list(shape))


# ------------------------------------------------------------------------------ SignSGD
def sign_compress(grad):
    from .signbits import sign_pack

    g = _flat(grad)
    lay = layout_for([(g.numel(),)])
    words = torch.empty(lay.n_words, dtype=torch.int64, device=g.device)
    sign_pack(g, lay, words)
    return words


def sign_decompress(words, shape):
    from .signbits import sign_unpack

    n = _numel(shape)
    lay = layout_for([(n,)])
    rows = words.reshape(-1, lay.n_words).contiguous()
    base = rows.view(torch.uint8).reshape(-1)
    out = torch.empty(n, dtype=torch.float32, device=words.device)
    sign_unpack(base, lay.n_words * 8, 0, 0, rows.shape[0], lay, out, vote=True)
    return out.view(list(shape))


# ------------------------------------------------------------------------------ QSGD
def qsgd_compress(grad, levels, seed):
    from .quant import qsgd_quantize

    g = _flat(grad)
    lay = layout_for([(g.numel(),)])
    norm = torch.linalg.vector_norm(g).reshape(1).float()
    codes = torch.empty(g.numel(), dtype=torch.int8 if levels < 128 else torch.int16, device=g.device)
    qsgd_quantize(g, lay, norm, int(levels), int(seed), codes)
    return codes, norm


def qsgd_decompress(codes, norms, levels, shape):
    from .quant import qsgd_aggregate

    n = _numel(shape)
    lay = layout_for([(n,)])
    W = norms.numel()
    cb = codes.element_size() * n
    row = -(-(cb + 4) // 16) * 16  # [codes | norm] rows, 16-B granular
    base = torch.zeros(W, row, dtype=torch.uint8, device=codes.device)
    base[:, :cb].copy_(codes.reshape(W, n).contiguous().view(torch.uint8))
    base[:, cb:cb + 4].copy_(norms.reshape(W, 1).float().contiguous().view(torch.uint8))
    out = torch.empty(n, dtype=torch.float32, device=codes.device)
    qsgd_aggregate(base.view(-1), row, 0, cb, codes.dtype, W, int(levels), lay, out, 1.0)
    return out.view(list(shape))


# ------------------------------------------------------------------------------ Natural
def natural_compress(grad, seed):
    from .quant import natural_encode

    g = _flat(grad)
    codes = torch.empty(g.numel(), dtype=torch.uint8, device=g.device)
    natural_encode(g, int(seed), codes)
    return codes


def natural_decompress(codes, shape):
    from .quant import natural_aggregate

    n = _numel(shape)
    rows = codes.reshape(-1, n).contiguous()
    out = torch.empty(n, dtype=torch.float32, device=codes.device)
    natural_aggregate(rows.view(-1), n, rows.shape[0], out, 1.0)
    return out.view(list(shape))


_IMPLS = {name: globals()[name] for name in _SCHEMAS}


def _fake_kernels():
    """Python fake kernels (only when the native library -- which carries the C++ Meta kernels --
    is unavailable)."""
    def zeros_like_shape(shape, like, dtype=torch.float32):
        return like.new_empty(list(shape), dtype=dtype)

    return {
        "topk_compress": lambda g, r, ratio, beta=1.0, gamma=1.0: (
            g.new_empty(k_of(g.numel(), ratio)), g.new_empty(k_of(g.numel(), ratio), dtype=torch.int32),
            torch.empty_like(g)),
        "sparse_decompress": lambda v, i, shape, scale=1.0: zeros_like_shape(shape, v),
        "randomk_compress": lambda g, ratio, seed: g.new_empty(k_of(g.numel(), ratio)),
        "randomk_decompress": lambda v, shape, ratio, seed, scale=1.0: zeros_like_shape(shape, v),
        "sign_compress": lambda g: g.new_empty((g.numel() + 63) // 64, dtype=torch.int64),
        "sign_decompress": lambda w, shape: zeros_like_shape(shape, w),
        "qsgd_compress": lambda g, levels, seed: (
            g.new_empty(g.numel(), dtype=torch.int8 if levels < 128 else torch.int16), g.new_empty(1)),
        "qsgd_decompress": lambda c, nrm, levels, shape: zeros_like_shape(shape, nrm),
        "natural_compress": lambda g, seed: g.new_empty(g.numel(), dtype=torch.uint8),
        "natural_decompress": lambda c, shape: zeros_like_shape(shape, c),
    }


def register() -> None:
    """Register the CUDA (native launchers) and CPU (reference path) kernels of every ``grace``
    op; idempotent."""
    global _LIB
    if _LIB is not None:
        return
    native = _native.available()  # loading grace_amd/_C.so runs its TORCH_LIBRARY(grace) block
    if native and hasattr(torch.ops.grace, "topk_compress"):
        lib = torch.library.Library("grace", "IMPL")
    else:  # no native library: the schemas + Python fake kernels
        lib = torch.library.Library("grace", "DEF")
        for schema in _SCHEMAS.values():
            lib.define(schema)
        for name, fk in _fake_kernels().items():
            torch.library.register_fake(f"grace::{name}", fk, lib=lib)
    for name, fn in _IMPLS.items():
        lib.impl(name, fn, "CPU")
        lib.impl(name, fn, "CUDA")
    _LIB = lib


def ops() -> List[str]:
    return sorted(_SCHEMAS)


__all__ = ["register", "ops", "k_of"] + sorted(_SCHEMAS)
