"""Property tests (hypothesis) over shapes the hand-written kernels find awkward: n < 64,
n = 2^k +- 1, one-element segments, many segments per bucket, heavy ties.

CPU runs check the PyTorch path; the ``gpu`` variants run the same properties through the HIP
kernels (survey 4, test plan item 2)."""
import math

import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from grace_amd import compressor as Z
from grace_amd.core import register_layout
from grace_amd.ops.layout import SegmentLayout

SIZES = st.one_of(st.integers(1, 70), st.sampled_from([63, 64, 65, 127, 128, 129, 255, 257, 1023, 1025, 8191,
                                                      8193, 16385]))
LAYOUTS = st.lists(SIZES, min_size=1, max_size=6)
SETTINGS = dict(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])


def _bucket(sizes, seed, ties=False, name="prop"):
    g = torch.Generator().manual_seed(seed)
    ts = [torch.randn(n, generator=g) for n in sizes]
    if ties:
        ts = [torch.round(t * 2) / 2 for t in ts]  # few distinct magnitudes -> many ties
    lay = SegmentLayout.from_tensors(ts)
    register_layout(name, lay)
    return torch.cat(ts), lay


def _check_topk(x, lay, ratio, dev):
    c = Z.TopKCompressor(ratio)
    payload, ctx = c.compress(x.to(dev), "prop")
    out = c.decompress(payload, ctx).cpu()
    for _, o, n in lay.segments():
        seg, got = x[o:o + n], out[o:o + n]
        k = max(1, int(n * ratio))
        kept = got != 0
        # exactly k kept unless kept values are themselves zero; kept values are exact
        assert int(kept.sum()) <= k
        assert torch.equal(got[kept], seg[kept])
        if kept.any() and (~kept).any():
            assert seg[kept].abs().min() >= seg[~kept].abs().max()


def _check_sign_roundtrip(x, lay, dev):
    c = Z.SignSGDCompressor()
    payload, ctx = c.compress(x.to(dev), "prop")
    out = c.decompress(payload, ctx).cpu()
    assert torch.equal(out, torch.where(x >= 0, 1.0, -1.0))


def _check_randomk(x, lay, ratio, dev):
    a, b = Z.RandomKCompressor(ratio), Z.RandomKCompressor(ratio)
    pa, ca = a.compress(x.to(dev), "prop")
    pb, cb = b.compress(x.to(dev), "prop")
    assert torch.equal(pa[0].cpu(), pb[0].cpu())  # same (name, step) -> same indices on every rank
    idx = a.indices(ca)
    assert idx.numel() == len(set(idx.tolist()))
    for (_, o, n), k in zip(lay.segments(), ca.ks):
        sel = idx[(idx >= o) & (idx < o + n)]
        assert sel.numel() == k


def _check_qsgd(x, lay, s, dev):
    c = Z.QSGDCompressor(s)
    payload, ctx = c.compress(x.to(dev), "prop")
    out = c.decompress(payload, ctx).cpu()
    for _, o, n in lay.segments():
        nrm = x[o:o + n].norm()
        assert ((out[o:o + n] - x[o:o + n]).abs() <= nrm / s * (1 + 1e-5) + 1e-6).all()


@given(LAYOUTS, st.integers(0, 10_000), st.sampled_from([0.01, 0.1, 0.5]), st.booleans())
@settings(**SETTINGS)
def test_topk_properties_cpu(sizes, seed, ratio, ties):
    x, lay = _bucket(sizes, seed, ties)
    _check_topk(x, lay, ratio, "cpu")


@given(LAYOUTS, st.integers(0, 10_000))
@settings(**SETTINGS)
def test_sign_roundtrip_cpu(sizes, seed):
    x, lay = _bucket(sizes, seed)
    _check_sign_roundtrip(x, lay, "cpu")


@given(LAYOUTS, st.integers(0, 10_000), st.sampled_from([0.05, 0.3]))
@settings(**SETTINGS)
def test_randomk_properties_cpu(sizes, seed, ratio):
    x, lay = _bucket(sizes, seed)
    _check_randomk(x, lay, ratio, "cpu")


@given(LAYOUTS, st.integers(0, 10_000), st.sampled_from([1, 4, 7, 64, 127]))
@settings(**SETTINGS)
def test_qsgd_error_bound_cpu(sizes, seed, s):
    x, lay = _bucket(sizes, seed)
    _check_qsgd(x, lay, s, "cpu")


# ------------------------------------------------------------------ same properties on the HIP kernels
@pytest.mark.gpu
@given(LAYOUTS, st.integers(0, 10_000), st.sampled_from([0.01, 0.1, 0.5]), st.booleans())
@settings(**SETTINGS)
def test_topk_properties_gpu(sizes, seed, ratio, ties):
    x, lay = _bucket(sizes, seed, ties)
    _check_topk(x, lay, ratio, "cuda")


@pytest.mark.gpu
@given(LAYOUTS, st.integers(0, 10_000))
@settings(**SETTINGS)
def test_sign_roundtrip_gpu(sizes, seed):
    x, lay = _bucket(sizes, seed)
    _check_sign_roundtrip(x, lay, "cuda")


@pytest.mark.gpu
@given(LAYOUTS, st.integers(0, 10_000), st.sampled_from([0.05, 0.3]))
@settings(**SETTINGS)
def test_randomk_properties_gpu(sizes, seed, ratio):
    x, lay = _bucket(sizes, seed)
    _check_randomk(x, lay, ratio, "cuda")


@pytest.mark.gpu
@given(LAYOUTS, st.integers(0, 10_000), st.sampled_from([1, 4, 7, 64, 127]))
@settings(**SETTINGS)
def test_qsgd_error_bound_gpu(sizes, seed, s):
    x, lay = _bucket(sizes, seed)
    _check_qsgd(x, lay, s, "cuda")
