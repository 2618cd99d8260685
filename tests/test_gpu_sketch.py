"""GPU: the native multi-rank radix select of the Sketch codec (csrc/kernels/quantile.hip).

The selected quantile edges must equal the sort-based PyTorch path bit for bit (exact order
statistics, torch's interpolation rounding), on distributions that stress the radix digits:
heavy ties, all-equal segments, signed zeros, tiny segments (n < q), wide dynamic range; the
full codec must equal the CPU path, and a captured graph must replay it.
"""
import pytest
import torch

from grace_amd import compressor as Z
from grace_amd.compressor.sketch import native_quantile_edges, segmented_quantile_edges
from grace_amd.core import register_layout
from grace_amd.ops import _native
from grace_amd.ops.layout import SegmentLayout

pytestmark = pytest.mark.gpu


def _segments(seed=0):
    g = torch.Generator().manual_seed(seed)
    return [
        torch.randn(100003, generator=g),
        torch.randint(-5, 6, (40000,), generator=g).float(),          # heavy ties
        torch.full((777,), 0.125),                                     # all equal
        torch.tensor([0.0, -0.0] * 50),                                # signed zeros
        torch.randn(1, generator=g),                                   # n = 1
        torch.randn(37, generator=g),                                  # n < q
        torch.randn(3000, generator=g) * torch.logspace(-30, 30, 3000),  # wide exponents
        -torch.rand(65536 * 3 + 5, generator=g),                       # all negative, > 1 chunk
        torch.randn(257, 129, generator=g).flatten() * 1e-3,
    ]


@pytest.mark.parametrize("q", [64, 16, 127, 255, 512])
def test_native_edges_equal_sort_edges(q):
    assert _native.available()
    segs = _segments()
    x = torch.cat(segs).cuda()
    lay = SegmentLayout.from_tensors(segs)
    got = native_quantile_edges(x, lay, q)
    ref = segmented_quantile_edges(x, lay, q)
    assert got is not None
    assert torch.equal(got, ref), (got - ref).abs().max()
    # second call: the kernels left their histograms clean
    got2 = native_quantile_edges(x * 2, lay, q)
    assert torch.equal(got2, segmented_quantile_edges(x * 2, lay, q))


def test_sketch_codec_gpu_matches_cpu():
    segs = _segments(1)
    flat = torch.cat(segs)
    lay = SegmentLayout.from_tensors(segs)
    register_layout("sk_bucket", lay)
    comp_c, comp_g = Z.SketchCompressor(64), Z.SketchCompressor(64)
    pc, cc = comp_c.compress(flat, "sk_bucket")
    pg, cg = comp_g.compress(flat.cuda(), "sk_bucket")
    assert torch.equal(pg[0].cpu(), pc[0])  # bin codes
    torch.testing.assert_close(pg[1].cpu(), pc[1], rtol=1e-5, atol=1e-6)  # bin means (atomic sum order)
    torch.testing.assert_close(comp_g.decompress(pg, cg).cpu(), comp_c.decompress(pc, cc), rtol=1e-5, atol=1e-6)
    # the encode's per-segment totals are a persistent workspace that the last block of every
    # segment turns into means and re-zeroes, and the bin sums are int64 fixed point (order-
    # independent): a second call is bit-identical, and scaling by 4 scales every mean exactly
    m1 = pg[1].clone()
    pg2, _ = comp_g.compress(flat.cuda(), "sk_bucket")
    assert torch.equal(pg2[1], m1)
    pg3, _ = comp_g.compress(flat.cuda() * 4, "sk_bucket")
    assert torch.equal(pg3[1], m1 * 4)


def test_sketch_graph_replay_equals_eager():
    segs = _segments(2)
    lay = SegmentLayout.from_tensors(segs)
    register_layout("sk_graph", lay)
    x = torch.cat(segs).cuda()
    comp = Z.SketchCompressor(64)
    eager = comp.decompress(*comp.compress(x, "sk_graph")).clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        comp.decompress(*comp.compress(x, "sk_graph"))  # warm the caches outside capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = comp.decompress(*comp.compress(x, "sk_graph"))
    x.mul_(-1.0)
    g.replay()
    torch.cuda.synchronize()
    got = out.clone()  # eager calls below may reuse the static output buffer
    ref = comp.decompress(*comp.compress(x.clone(), "sk_graph")).clone()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    assert not torch.equal(got, eager)


@pytest.mark.parametrize("q", [255, 512])
def test_sketch_large_q_codec_and_graph(q):
    """q >= 128 (uint16/int16 bins, batched native select): CPU parity and graph capture."""
    from grace_amd.parallel.graph import graph_safe
    from grace_amd import grace_from_params
    from grace_amd.parallel.comm import LocalComm

    assert graph_safe(grace_from_params({"compressor": "sketch", "quantiles": q}, comm=LocalComm())) is None
    segs = _segments(3)
    flat = torch.cat(segs)
    lay = SegmentLayout.from_tensors(segs)
    register_layout(f"skq{q}", lay)
    comp_c, comp_g = Z.SketchCompressor(q), Z.SketchCompressor(q)
    pc, cc = comp_c.compress(flat, f"skq{q}")
    pg, cg = comp_g.compress(flat.cuda(), f"skq{q}")
    assert pg[0].dtype == (torch.int16 if q >= 256 else torch.uint8) and torch.equal(pg[0].cpu(), pc[0])
    torch.testing.assert_close(comp_g.decompress(pg, cg).cpu(), comp_c.decompress(pc, cc), rtol=1e-5, atol=1e-6)
    x = flat.cuda()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        comp_g.decompress(*comp_g.compress(x, f"skq{q}"))
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = comp_g.decompress(*comp_g.compress(x, f"skq{q}"))
    x.mul_(0.5)
    g.replay()
    torch.cuda.synchronize()
    got = out.clone()
    ref = comp_g.decompress(*comp_g.compress(x.clone(), f"skq{q}")).clone()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("q", [1024, 1500, 4096])
def test_large_q_native_codec_matches_sort_path(q):
    """q > 1024 (the reference's uint16 bins go to 65535; tensorflow/compressor/sketch.py:22-27):
    the batched native select gives the sort path's edges bit for bit, the global-accumulator
    encode gives its bin codes bit for bit and its means to fp32 summation order, deterministic
    across calls, and the whole codec replays from a captured graph (no sort, no host read)."""
    from grace_amd.parallel.graph import graph_safe
    from grace_amd import grace_from_params

    segs = _segments(3)
    flat = torch.cat(segs)
    lay = SegmentLayout.from_tensors(segs)
    name = f"sk_big{q}"
    register_layout(name, lay)
    x = flat.cuda()
    assert torch.equal(native_quantile_edges(x, lay, q), segmented_quantile_edges(x, lay, q))
    comp_c, comp_g = Z.SketchCompressor(q), Z.SketchCompressor(q)
    pc, cc = comp_c.compress(flat, name)
    pg, cg = comp_g.compress(x, name)
    assert pg[0].dtype == torch.int16
    assert torch.equal(pg[0].cpu(), pc[0])  # bin codes
    torch.testing.assert_close(pg[1].cpu(), pc[1], rtol=1e-5, atol=1e-6)
    m1 = pg[1].clone()
    assert torch.equal(comp_g.compress(x, name)[0][1], m1)  # fixed-point sums: order-independent
    torch.testing.assert_close(comp_g.decompress(pg, cg).cpu(), comp_c.decompress(pc, cc), rtol=1e-5, atol=1e-6)
    grc = grace_from_params({"compressor": "sketch", "quantiles": q, "memory": "none", "communicator": "allgather",
                             "world_size": 1})
    assert graph_safe(grc) is None
    eager = grc.step(x.clone(), name).clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        grc.step(x.clone(), name)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    xs = x.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = grc.step(xs, name)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, eager)
