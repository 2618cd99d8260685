"""GPU numerics: every native compressor kernel vs the PyTorch fp32 reference path.

Deterministic codecs must match the CPU/PyTorch path (bit-exact or to fp32 rounding);
stochastic ones (QSGD, TernGrad, Natural) are checked for their error bounds and
unbiasedness, on the GPU path that runs the HIP kernels.
"""
import math
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(__file__))
import oracles as O  # noqa: E402
from grace_amd import compressor as Z  # noqa: E402
from grace_amd import memory as M  # noqa: E402
from grace_amd.communicator import Allgather, Allreduce  # noqa: E402
from grace_amd.core import register_layout  # noqa: E402
from grace_amd.ops import _native  # noqa: E402
from grace_amd.ops.layout import SegmentLayout  # noqa: E402
from grace_amd.parallel.comm import LocalComm  # noqa: E402

pytestmark = pytest.mark.gpu

SHAPES = [(10, 7), (64,), (3, 3, 3, 3), (1,), (129,), (257, 129), (4096,), (100003,)]


def _bucket(seed=0):
    g = torch.Generator().manual_seed(seed)
    ts = [torch.randn(*s, generator=g) for s in SHAPES]
    flat = torch.cat([t.flatten() for t in ts])
    lay = SegmentLayout.from_tensors(ts)
    register_layout("gpu_bucket", lay)
    return flat, lay


def _rt(comp, x, name="gpu_bucket"):
    payload, ctx = comp.compress(x, name)
    return comp.decompress(payload, ctx)


def test_native_library_loaded():
    assert _native.available(), "grace_amd/_C.so must load on the GPU box"
    assert "gfx950" in _native.lib().build_info()


@pytest.mark.parametrize("make", [
    lambda: Z.TopKCompressor(0.05),
    lambda: Z.SignSGDCompressor(),
    lambda: Z.EFSignSGDCompressor(0.1),
    lambda: Z.OneBitCompressor(),
    lambda: Z.U8bitCompressor(),
    lambda: Z.ThresholdCompressor(1.5),
])
def test_deterministic_codecs_match_torch(make):
    flat, lay = _bucket()
    cpu = _rt(make(), flat)
    gpu = _rt(make(), flat.cuda())
    torch.testing.assert_close(gpu.cpu(), cpu, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("make", [
    lambda: Z.TopKCompressor(0.05),
    lambda: Z.SignSGDCompressor(),
    lambda: Z.SignumCompressor(0.9),
    lambda: Z.EFSignSGDCompressor(0.1),
    lambda: Z.OneBitCompressor(),
    lambda: Z.U8bitCompressor(),
    lambda: Z.RandomKCompressor(0.05),
])
def test_fused_residual_matches_torch(make):
    """Fused error-feedback kernels == PyTorch path over 3 steps (residuals too)."""
    outs = {}
    for dev in ("cpu", "cuda"):
        grc = Allgather(make(), M.ResidualMemory(beta=0.9, gamma=1.0), comm=LocalComm())
        res = []
        for s in range(3):
            flat, _ = _bucket(seed=s)
            res.append(grc.step(flat.to(dev), "gpu_bucket").cpu())
        res.append(grc.memory.residuals["gpu_bucket"].cpu())
        outs[dev] = res
    for a, b in zip(outs["cpu"], outs["cuda"]):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-5)


def test_randomk_same_indices_cpu_gpu():
    flat, lay = _bucket()
    a = _rt(Z.RandomKCompressor(0.1), flat)
    b = _rt(Z.RandomKCompressor(0.1), flat.cuda()).cpu()
    torch.testing.assert_close(a, b)


def test_qsgd_gpu_bounds_unbiased():
    flat, lay = _bucket()
    x = flat.cuda()
    c = Z.QSGDCompressor(64)
    acc = torch.zeros_like(x)
    n = 100
    for _ in range(n):
        d = _rt(c, x)
        acc += d
    # per-segment bound: |dec - x| <= ||seg||/s
    for (i, o, k) in lay.segments():
        seg = flat[o:o + k]
        assert (d[o:o + k].cpu() - seg).abs().max() <= seg.norm() / 64 * (1 + 1e-4) + 1e-7
    # unbiased: per-element error of the n-sample mean has std <= step/(2 sqrt(n)), so
    # E|err| <= 0.4 step/sqrt(n); and the signed errors average out (no systematic bias)
    big = slice(lay.offsets[-2], lay.offsets[-1])
    step = flat[big].norm().item() / 64
    err = (acc[big] / n - x[big]).cpu()
    assert err.abs().mean() <= 0.45 * step / n ** 0.5
    assert abs(err.mean().item()) <= 5 * 0.5 * step / (n * err.numel()) ** 0.5


def test_terngrad_gpu():
    flat, lay = _bucket()
    x = flat.cuda()
    c = Z.TernGradCompressor()
    d = _rt(c, x).cpu()
    for (i, o, k) in lay.segments():
        seg = flat[o:o + k]
        sc = O.terngrad_scalar(seg)
        vals = set(torch.unique(d[o:o + k] / sc).round().tolist()) if sc > 0 else {0.0}
        assert vals <= {-1.0, 0.0, 1.0}


def test_natural_gpu_power_of_two():
    flat, _ = _bucket()
    d = _rt(Z.NaturalCompressor(), flat.cuda()).cpu()
    lo, hi = O.natural_decode_range(flat)
    a = d.abs()
    assert torch.all(torch.isclose(a, lo) | torch.isclose(a, hi))


def test_dgc_gpu_selects_about_ratio():
    flat, lay = _bucket()
    c = Z.DgcCompressor(0.01)
    payload, ctx = c.compress(flat.cuda(), "gpu_bucket")
    big = lay.numels[-1]
    hdr, vals, idx = (t.cpu() for t in payload)
    n = min(int(hdr[0]), vals.numel())
    assert int(hdr[0]) <= vals.numel(), "capacity overflow on N(0,1) data"
    idx = idx[:n].long()
    n_big = ((idx >= lay.offsets[-2]) & (idx < lay.offsets[-1])).sum().item()
    assert 0.5 * 0.01 * big <= n_big <= 1.5 * 0.01 * big
    assert torch.equal(vals[:n], flat[idx])


@pytest.mark.parametrize("rank", [1, 2, 4])
def test_powersgd_kernels_match_torch(rank):
    from grace_amd.ops import powersgd as PS

    g = torch.Generator().manual_seed(3)
    shapes = [(300, 257), (64, 3, 3, 3), (1000,), (4096, 1100)]
    ts = [torch.randn(*s, generator=g) for s in shapes]
    flat = torch.cat([t.flatten() for t in ts])
    lay = SegmentLayout.from_tensors(ts)
    plan = PS.plan_for(lay, rank)
    q = torch.randn(plan.q_total, generator=g)
    xg, qg = flat.cuda(), q.cuda()
    p_ref = PS.mq(flat, q, plan)
    p_gpu = PS.mq(xg, qg, plan)
    # fp32 sums of up to 4096 terms in a different order: compare against the output scale
    torch.testing.assert_close(p_gpu.cpu(), p_ref, rtol=1e-4, atol=2e-6 * p_ref.abs().max().item())
    q_ref = PS.mtp(flat, p_ref, plan)
    q_gpu = PS.mtp(xg, p_ref.cuda(), plan)
    torch.testing.assert_close(q_gpu.cpu(), q_ref, rtol=1e-4, atol=2e-6 * q_ref.abs().max().item())
    a = p_ref.clone()
    PS.orthogonalize(a, plan, "p")
    b = p_ref.cuda()
    PS.orthogonalize(b, plan, "p")
    torch.testing.assert_close(b.cpu(), a, rtol=1e-4, atol=1e-4)
    out_ref = torch.zeros(lay.total)
    PS.pqt(a, q_ref, plan, out_ref)
    out_gpu = torch.zeros(lay.total, device="cuda")
    PS.pqt(a.cuda(), q_ref.cuda(), plan, out_gpu)
    torch.testing.assert_close(out_gpu.cpu(), out_ref, rtol=1e-4, atol=1e-4)


def test_powersgd_allreduce_gpu_step():
    x = torch.randn(512, 300, device="cuda")
    grc = Allreduce(Z.PowerSGDCompressor(rank=4), M.PowerSGDMemory(compress_rank=4), comm=LocalComm())
    out = grc.step(x, "w")
    assert torch.isfinite(out).all()
    # rank-4 approximation never exceeds the input energy
    assert out.norm() <= x.norm() * 1.0001


def test_segment_stats_gpu():
    from grace_amd.ops import segstats as S

    flat, lay = _bucket()
    a = S.segment_stats(flat, lay)
    b = S.segment_stats(flat.cuda(), lay).cpu()
    torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-4)


def test_gram_orthonormalize_orthogonal_and_rank_deficient():
    from grace_amd.ops import powersgd as PS

    g = torch.Generator().manual_seed(5)
    shapes = [(25088, 64), (300, 40), (7, 5)]
    lay = SegmentLayout.from_tensors([torch.empty(s) for s in shapes])
    plan = PS.plan_for(lay, 4)
    p = torch.randn(plan.p_total, generator=g)
    # ill-conditioned first matrix (column scales 1 .. 1e-3) and an exactly dependent column
    (xo, n, m, r, po, qo) = plan.mats[0]
    p[po:po + n * r].view(n, r).mul_(torch.tensor([1.0, 1e-1, 1e-2, 1e-3]))
    (xo, n, m, r, po, qo) = plan.mats[1]
    v = p[po:po + n * r].view(n, r)
    v[:, 2] = 2.0 * v[:, 0]
    b = p.cuda()
    PS.orthogonalize(b, plan, "p")
    b = b.cpu()
    for i, (xo, n, m, r, po, qo) in enumerate(plan.mats):
        a = b[po:po + n * r].view(n, r).double()
        gram = a.t() @ a
        if i == 1:  # dependent column -> (near) zero, the others orthonormal
            keep = [0, 1, 3]
            assert a[:, 2].norm() < 1e-3 or abs(a[:, 2].norm() - 1) < 1e-3
            gram = gram[keep][:, keep]
        assert (gram - torch.eye(gram.shape[0], dtype=torch.float64)).abs().max() < 1e-5
    # same span / signs as the reference MGS on a well-conditioned matrix
    ref = p.clone()
    PS.orthogonalize(ref, plan, "p")
    (xo, n, m, r, po, qo) = plan.mats[2]
    torch.testing.assert_close(b[po:po + n * r], ref[po:po + n * r], rtol=1e-4, atol=1e-5)


def test_powersgd_fused_memory_gpu_matches_cpu_unfused(monkeypatch):
    """Fused GPU PowerSGD (+ memory) == unfused CPU PowerSGD with the SAME Q: the CPU path's Q
    is drawn by the native Philox generator with the host-mixed seed, which is bit-identical to
    the GPU's (base seed, device step) draw (tests/test_gpu_graph_rng.py)."""
    from grace_amd.core import register_layout
    from grace_amd.ops import powersgd as PS

    real = PS.randn_shared

    def shared_q(n, seed, device, step=None, zero=None):
        if torch.device(device).type == "cpu":
            if zero is not None:
                zero.zero_()
            return real(n, seed, "cuda").cpu()
        return real(n, seed, device, step=step, zero=zero)

    monkeypatch.setattr(PS, "randn_shared", shared_q)

    class Unfused(M.PowerSGDMemory):
        pass

    shapes = [(512, 300), (64,), (32, 16, 3, 3), (10,)]
    register_layout("psgd_gpu", SegmentLayout.from_tensors([torch.empty(s) for s in shapes]))
    outs = {}
    for dev, mem_cls in (("cuda", M.PowerSGDMemory), ("cpu", Unfused)):
        mem = mem_cls(compress_rank=4)
        grc = Allreduce(Z.PowerSGDCompressor(rank=4), mem, comm=LocalComm())
        res = []
        for s in range(3):
            gen = torch.Generator().manual_seed(s)
            x = torch.cat([torch.randn(*sh, generator=gen).flatten() for sh in shapes])
            res.append(grc.step(x.to(dev), "psgd_gpu").cpu())
        sd = mem.state_dict()["residuals"]["psgd_gpu"].reshape(-1).cpu()  # materialised copy
        mem.materialize()  # the GPU memory defers its residual update (PowerSGDMemory.lazy)
        res.append(mem.residuals["psgd_gpu"].reshape(-1).cpu())
        assert torch.equal(sd, res[-1])
        outs[dev] = res
    for a, b in zip(outs["cuda"], outs["cpu"]):  # 3 decoded steps + the final residual
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)


def test_segment_stats_large_unaligned_segment():
    from grace_amd.ops import segstats as S

    g = torch.Generator().manual_seed(9)
    ts = [torch.randn(3, generator=g), torch.randn(5_000_011, generator=g), torch.randn(77, generator=g)]
    lay = SegmentLayout.from_tensors(ts)
    flat = torch.cat(ts)
    r = torch.randn(flat.numel(), generator=g)
    ref = torch.stack([torch.stack([t.double().sum(), (t.double() ** 2).sum(), t.abs().max().double(),
                                    t.double().abs().sum(), t.double().clamp(max=0).sum(),
                                    (t < 0).sum().double()]) for t in ts]).float()
    b = S.segment_stats(flat.cuda(), lay).cpu()  # 16-B aligned base: float4 body
    torch.testing.assert_close(b, ref, rtol=1e-5, atol=1e-3)
    shifted = torch.cat([torch.zeros(1), flat]).cuda()[1:]  # 4-B offset base: scalar path
    torch.testing.assert_close(S.segment_stats(shifted, lay).cpu(), ref, rtol=1e-5, atol=1e-3)
    # fused compensate (x = 0.5 r + 2 g stored to xout) through the misaligned-view path
    xg = torch.empty_like(flat).cuda()
    S.segment_stats(flat.cuda(), lay, r=r.cuda(), r_valid=True, beta=0.5, gamma=2.0, xout=xg)
    torch.testing.assert_close(xg.cpu(), 0.5 * r + 2.0 * flat, rtol=1e-6, atol=1e-6)


def test_inceptionn_native_bit_exact():
    """HIP INCEPTIONN encode/decode == the PyTorch codec bit for bit (payload and result),
    including W=3 rank-ordered aggregation."""
    g = torch.Generator().manual_seed(11)
    n = 300_001  # several tiles plus a ragged tail
    x = torch.randn(n, generator=g) * torch.logspace(-12, 1, n)[torch.randperm(n, generator=g)]
    x[::97] = 0.0
    register_layout("inc_bucket", SegmentLayout.from_tensors([x]))
    comp = Z.INCEPTIONNCompressor(2e-10)
    pc, ctx_c = comp.compress(x, "inc_bucket")
    pg, ctx_g = comp.compress(x.cuda(), "inc_bucket")
    for a, b in zip(pc, pg):
        assert a.dtype == b.dtype and a.numel() == b.numel()
    # header (class totals) and codes bit-exact; the value stream up to its used bytes (the
    # capacity tail past them is never read and left unwritten on the GPU)
    assert torch.equal(pc[0], pg[0].cpu()) and torch.equal(pc[2], pg[2].cpu())
    _, n8, n16, n32 = pc[0].tolist()
    used = 4 * n32 + 2 * n16 + n8
    assert torch.equal(pc[1][:used], pg[1][:used].cpu())
    others = [comp.compress(x * s, "inc_bucket")[0] for s in (0.5, -3.0)]
    ref = comp.decompress_aggregate([pc] + others, ctx_c, 3)
    got = comp.decompress_aggregate([pg] + [[t.cuda() for t in o] for o in others], ctx_g, 3)
    assert torch.equal(got.cpu(), ref)


def test_inceptionn_capacity_drops_lowest_classes_first():
    """capacity < 1: the 8-bit class is dropped before the 16-bit one; GPU == CPU oracle."""
    g = torch.Generator().manual_seed(12)
    n = 100_000
    x = torch.randn(n, generator=g) * torch.logspace(-9, 1, n)[torch.randperm(n, generator=g)]
    register_layout("inc_cap", SegmentLayout.from_tensors([x]))
    full = Z.INCEPTIONNCompressor(2e-10)
    _, n8, n16, n32 = full.compress(x, "inc_cap")[0][0].tolist()
    cap = (4 * n32 + 2 * n16 + n8 // 2) / (4 * n)  # room for v32 + v16, not for all of v8
    comp = Z.INCEPTIONNCompressor(2e-10, capacity=cap)
    pc, ctx_c = comp.compress(x, "inc_cap")
    pg, ctx_g = comp.compress(x.cuda(), "inc_cap")
    assert torch.equal(pc[2], pg[2].cpu())
    codes = ((pc[2].long().unsqueeze(1) >> torch.tensor([0, 2, 4, 6])) & 3).view(-1)[:n]
    assert int((codes == 1).sum()) == 0 and int((codes == 2).sum()) == n16 and int((codes == 3).sum()) == n32
    torch.testing.assert_close(comp.decompress(pg, ctx_g).cpu(), comp.decompress(pc, ctx_c), rtol=0, atol=0)


def test_adaq_native_properties():
    """HIP Adaq: per (segment, side) group the indices lie in the segment with the right sign,
    the sent mean is the mean of the selected values, the count is near ratio * side size,
    and decompress scatters the means (stochastic sampling: checked by properties)."""
    import math

    g = torch.Generator().manual_seed(21)
    shapes = [(1000, 50), (7,), (200_003,), (64, 3, 3, 3)]
    ts = [torch.randn(*s, generator=g) for s in shapes]
    ts[1] = ts[1].abs()  # a segment with no negative side
    lay = SegmentLayout.from_tensors(ts)
    register_layout("adaq_bucket", lay)
    x = torch.cat([t.flatten() for t in ts])
    comp = Z.AdaqCompressor(0.05)
    payload, ctx = comp.compress(x.cuda(), "adaq_bucket")
    m, cnt, ix = (t.cpu() for t in payload)
    assert ix.numel() == comp._cap(lay) >= int(cnt.sum())  # fixed capacity, in-band counts
    ix = ix[: int(cnt.sum())]
    pos = 0
    for s, o, n in lay.segments():
        seg = x[o:o + n]
        for side in (0, 1):
            c = int(cnt[2 * s + side])
            idx = ix[pos:pos + c].long()
            pos += c
            assert ((idx >= o) & (idx < o + n)).all()
            v = x[idx]
            assert (v > 0).all() if side == 0 else (v < 0).all()
            n_side = int((seg > 0).sum() if side == 0 else (seg < 0).sum())
            if c:
                torch.testing.assert_close(m[2 * s + side], v.mean(), rtol=1e-5, atol=1e-6)
                assert len(set(idx.tolist())) == c
            else:
                assert m[2 * s + side] == 0
            target = math.ceil(0.05 * n_side)
            if n_side >= 1000:
                assert 0.7 * target <= c <= 1.3 * target, (s, side, c, target)
            if n_side == 0:
                assert c == 0
    dec = comp.decompress([t.cuda() for t in payload], ctx).cpu()
    ref = torch.zeros_like(x)
    ref[ix.long()] = torch.repeat_interleave(m, cnt.long())
    torch.testing.assert_close(dec, ref)


@pytest.mark.parametrize("rank", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("passes_for", ["p", "q"])
def test_gram_orthonormalize_ranks_gpu(rank, passes_for):
    """One-launch small-rank form (r <= 4) and the MFMA three-kernel form (r > 4): columns come
    out orthonormal and span-equal to the reference MGS for every matrix of the bucket."""
    from grace_amd.ops import powersgd as PS

    g = torch.Generator().manual_seed(11 + rank)
    shapes = [(25088, 300), (513, 40), (6, 9), (33, 2)]
    lay = SegmentLayout.from_tensors([torch.empty(s) for s in shapes])
    plan = PS.plan_for(lay, rank)
    total = plan.p_total if passes_for == "p" else plan.q_total
    a = torch.randn(total, generator=g)
    b = a.cuda()
    PS.orthogonalize(b, plan, passes_for)
    ref = a.clone()
    PS.orthogonalize(ref, plan, passes_for)
    b = b.cpu()
    for (xo, n, m, r, po, qo) in plan.mats:
        off, ln = (po, n) if passes_for == "p" else (qo, m)
        got = b[off:off + ln * r].view(ln, r).double()
        assert (got.t() @ got - torch.eye(r, dtype=torch.float64)).abs().max() < 1e-5
        torch.testing.assert_close(got.float(), ref[off:off + ln * r].view(ln, r), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("s,bits", [(1, 2), (3, 4), (7, 4)])
def test_qsgd_packed_codes_gpu(s, bits):
    """Native pack + packed-row decode (csrc/kernels/quant.hip qsgd_pack_kernel, PackedCode<B>)
    equals the int8-code native path bit for bit, and the CPU torch path's packing."""
    from grace_amd import compressor as Z

    class Unpacked(Z.QSGDCompressor):
        @property
        def pack_bits(self):
            return 0

    g = torch.Generator().manual_seed(5)
    x = torch.randn(100003, generator=g).cuda()
    cp, cu = Z.QSGDCompressor(s), Unpacked(s)
    tp, ctxp = cp.compress(x, "w")
    tu, ctxu = cu.compress(x, "w")
    assert tp[0].dtype == torch.uint8 and tp[0].numel() == (x.numel() * bits + 7) // 8
    torch.testing.assert_close(cp.decompress(tp, ctxp), cu.decompress(tu, ctxu), rtol=0, atol=0)
    # the packed bytes equal the torch reference packing of the same int8 codes
    from grace_amd.ops import quant as Q
    codes = tu[0][: x.numel()].cpu()
    ref_cpu = torch.zeros(tp[0].numel(), dtype=torch.uint8)
    Q.qsgd_pack(codes, s, bits, ref_cpu)
    assert torch.equal(tp[0].cpu(), ref_cpu)


def test_powersgd_rank_deficient_is_exact_gpu():
    """A full-rank-capable PowerSGD (rank >= min(n, m)) on a rank-DEFICIENT matrix (a zero row,
    e.g. dead ReLU units) must reproduce the matrix: the dependent column of P becomes zero in
    the native Gram MGS instead of normalised rounding noise."""
    from grace_amd import grace_from_params
    from grace_amd.parallel.comm import LocalComm

    torch.manual_seed(0)
    for shape, dead in (((4, 16), 2), ((3, 4), 1), ((8, 300), 5)):
        m = torch.randn(*shape, device="cuda") * 0.01
        m[dead, :] = 0
        g = grace_from_params({"compressor": "powersgd", "compress_rank": min(shape), "communicator": "allreduce"},
                              comm=LocalComm())
        out = g.step(m.clone(), "w")
        torch.cuda.synchronize()
        assert (out - m).abs().max() <= 1e-5 * m.abs().max(), shape


def test_dgc_tree_refinement_matches_sequential_rule():
    """the speculative tree refinement (3 steps per count pass) ends on exactly the thresholds the
    reference's sequential loop reaches (dist/compressor/dgc.py:27-36: x1.3 above 1.3 x target,
    x0.7 below 0.7 x target, at most 10 steps) from the same sampled start, in float32"""
    from grace_amd.ops import dgc as D
    from grace_amd.ops.dgc import _sizes
    from grace_amd.ops.topk import _workspace as topk_ws

    flat, lay = _bucket()
    x = flat.cuda() * torch.linspace(0.2, 3.0, flat.numel(), device="cuda")  # spread the scales
    dev = x.device
    cap = D.dgc_capacity(lay, 0.01, 2.0)
    D.dgc_select(x, lay, 0.01, 0.01, 10, 7, cap)
    ws = lay.cached(dev, "dgc_ws:0.01:0.01", lambda: None)
    ns, ks = _sizes(lay, 0.01, 0.01)
    slay = lay.cached(dev, "dgc_sample_layout:0.01", lambda: None)
    st = topk_ws(slay, ks, dev)["state"].cpu().view(-1, 2)
    thr0 = st[:, 0].contiguous().view(torch.float32)
    got = ws["thr"].cpu()
    xa = x.abs().cpu()
    f13, f07 = torch.tensor(1.3, dtype=torch.float32), torch.tensor(0.7, dtype=torch.float32)
    for s, (_, o, n) in enumerate(lay.segments()):
        t = thr0[s].clone()
        target = torch.tensor(n * 0.01, dtype=torch.float32)
        seg = xa[o:o + n]
        for _ in range(10):
            sel = (seg >= t).sum().to(torch.float32)
            if sel > f13 * target:
                t = t * f13
            elif sel < f07 * target:
                t = t * f07
            else:
                break
        assert torch.equal(got[s], t), (s, float(got[s]), float(t))


def test_dgc_fused_compensate_equals_compensate_then_select():
    """DgcMemory's compensate fused into the DGC selection (samples read v + (m u + g) on the fly,
    the first refinement count pass writes u and v) gives the compensate-pass-then-select
    payload and state bit for bit, over steps (first step: u = v = g)."""
    from grace_amd import compressor as Z
    from grace_amd import memory as M
    from grace_amd.core import register_layout
    from grace_amd.ops import _native
    from grace_amd.ops import dgc as D
    from grace_amd.ops.layout import SegmentLayout

    g0 = torch.Generator().manual_seed(11)
    shapes = [(512, 300), (1000,), (64, 3, 3, 3), (70001,)]
    lay = SegmentLayout.from_tensors([torch.empty(s) for s in shapes])
    register_layout("dgc_fuse", lay)
    comp_a, comp_b = Z.DgcCompressor(0.01), Z.DgcCompressor(0.01)
    mem_a, mem_b = M.DgcMemory(0.9, gradient_clipping=False), M.DgcMemory(0.9, gradient_clipping=False)
    C = _native.lib()
    for step in range(3):
        g = torch.randn(lay.total, generator=g0).cuda()
        pa, ca = comp_a.fused_compress(g.clone(), "dgc_fuse", mem_a)  # fused path
        # reference: explicit compensate pass, then the native selection on v
        gb = g.clone()
        u, v, first = mem_b.state_buffers("dgc_fuse", gb)
        C.dgc_compensate(gb, u, v, mem_b.momentum, first)
        cb = comp_b.ctx(gb, "dgc_fuse")
        pb, _ = comp_b._select(v, cb, "dgc_fuse", vmask=v, umask=u)
        torch.cuda.synchronize()
        ha, hb = pa[0].cpu(), pb[0].cpu()
        assert torch.equal(ha, hb), (step, ha, hb)
        k = min(int(ha[0]), int(ha[1]))
        ia, ib = pa[2][:k].long().cpu(), pb[2][:k].long().cpu()
        oa, ob = torch.argsort(ia), torch.argsort(ib)
        assert torch.equal(ia[oa], ib[ob]), step
        assert torch.equal(pa[1][:k].cpu()[oa], pb[1][:k].cpu()[ob]), step
        ua, va, _ = mem_a.state_buffers("dgc_fuse", g)
        assert torch.equal(ua, u) and torch.equal(va, v), step


@pytest.mark.parametrize("graphed", [False, True])
def test_powersgd_deferred_residual_bit_identical(graphed):
    """The deferred residual (r = M - s P Q^T formed inside the next P = M Q pass, with the float
    ops of the eager update) matches the eager residual update inside the decompress pass, step
    after step -- eager and HIP-graph-replayed -- and a mid-run state_dict (materialised copy)
    leaves the live deferred state untouched.  Not bitwise across the two runs: Q = M^T P sums its
    row strips with float atomics, so P / Q themselves differ in the last bit run to run."""
    import grace_amd.compressor.powersgd as CP
    from grace_amd.core import register_layout

    shapes = [(512, 300), (64,), (32, 16, 3, 3), (10,), (1000, 36)]
    register_layout("psgd_def", SegmentLayout.from_tensors([torch.empty(s) for s in shapes]))
    n = sum(math.prod(s) for s in shapes)
    xs = [torch.randn(n, generator=torch.Generator().manual_seed(s)).cuda() for s in range(6)]
    outs = {}
    for defer in (False, True):
        old = CP._DEFER_RESID
        CP._DEFER_RESID = defer
        try:
            mem = M.PowerSGDMemory(compress_rank=4)
            grc = Allreduce(Z.PowerSGDCompressor(rank=4), mem, comm=LocalComm())
            res = []
            if not graphed:
                for s, x in enumerate(xs):
                    res.append(grc.step(x, "psgd_def").clone())
                    if s == 2 and defer:
                        before = mem.residuals["psgd_def"].clone()
                        mem.state_dict()
                        assert torch.equal(before, mem.residuals["psgd_def"])
            else:
                buf = xs[0].clone()
                out = torch.empty_like(buf)
                st = torch.cuda.Stream()
                st.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(st):
                    for x in xs[:2]:  # warm-up: allocates residual / P-prev / arenas
                        buf.copy_(x)
                        out.copy_(grc.step(buf, "psgd_def"))
                        res.append(out.clone())
                torch.cuda.current_stream().wait_stream(st)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=st):
                    out.copy_(grc.step(buf, "psgd_def"))
                for x in xs[2:]:
                    buf.copy_(x)
                    g.replay()
                    res.append(out.clone())
            mem.materialize()
            res.append(mem.residuals["psgd_def"].reshape(-1).clone())
            outs[defer] = res
        finally:
            CP._DEFER_RESID = old
    for i, (a, b) in enumerate(zip(outs[False], outs[True])):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5, msg=lambda m, i=i: f"step {i}: {m}")


@pytest.mark.parametrize("max_iters", [0, 2, 5, 7, 10])
def test_dgc_scanned_compaction_exact(max_iters):
    """The DGC compaction places every chunk at a prefix-summed offset of the count pass's per-chunk
    counts (segments whose final threshold was never counted -- max_iters 0, or a walk that ended
    below the counted tree -- reserve slots with atomics after them): the payload holds exactly the
    entries |x| >= thr[segment], each once, the header counts them, and a too-small capacity keeps
    a duplicate-free subset with the full count in the header."""
    from grace_amd.ops import dgc as D

    flat, lay = _bucket()
    x = flat.cuda() * torch.linspace(0.2, 3.0, flat.numel(), device="cuda")
    dev = x.device
    seg_of = torch.repeat_interleave(torch.arange(lay.n_seg), torch.tensor(lay.numels))
    for capf in (2.0, 0.3):
        cap = D.dgc_capacity(lay, 0.01, capf)
        hdr, v, i = D.dgc_select(x, lay, 0.01, 0.01, max_iters, 7, cap)
        torch.cuda.synchronize()
        ws = lay.cached(dev, "dgc_ws:0.01:0.01", lambda: None)
        thr = ws["thr"].cpu()
        xa = x.cpu()
        sel = (xa.abs() >= thr[seg_of]).nonzero().flatten()
        count = int(hdr[0])
        assert count == sel.numel(), (capf, count, sel.numel())
        k = min(count, cap)
        got = i[:k].cpu().long()
        assert got.unique().numel() == k, "duplicate slots"
        assert torch.equal(xa[got], v[:k].cpu()), "value / index mismatch"
        if k == count:
            assert torch.equal(got.sort().values, sel), "selected set differs"
        else:
            assert bool(torch.isin(got, sel).all()), "entry below its threshold sent"
        if max_iters == 0:
            assert bool((ws["fnode"] < 0).all())


def test_dgc_sample_select_is_exact_kth_largest():
    """The one-launch sample select (one workgroup per segment, samples in LDS up to 24576 and
    re-read from memory beyond) starts the refinement at exactly the k'-th largest |sample| of
    every segment -- the reference's torch.topk(samples, k').values.min() (dgc.py:21-24)."""
    from grace_amd.ops import dgc as D
    from grace_amd.ops.dgc import _sizes

    shapes = [(3000, 1000), (512, 300), (1000,), (64, 3, 3, 3), (7,), (2, 2)]
    lay = SegmentLayout.from_tensors([torch.empty(s) for s in shapes])
    x = torch.randn(lay.total, generator=torch.Generator().manual_seed(4)).cuda()
    D.dgc_select(x, lay, 0.01, 0.01, 0, 11, D.dgc_capacity(lay, 0.01, 2.0))
    torch.cuda.synchronize()
    ws = lay.cached(x.device, "dgc_ws:0.01:0.01", lambda: None)
    ns, ks = _sizes(lay, 0.01, 0.01)
    assert max(ns) > 24576  # the memory-resident path runs too
    samp = ws["samples"].cpu()
    thr = ws["thr"].cpu()
    o = 0
    for s, (n_s, k) in enumerate(zip(ns, ks)):
        ref = torch.topk(samp[o:o + n_s].abs(), k).values.min()
        assert torch.equal(thr[s], ref), (s, float(thr[s]), float(ref))
        o += n_s


def test_powersgd_step_level_gpu_merged_launches_match_per_bucket_and_cpu():
    """Several buckets on the GPU: the step-level exchange (one M^T P launch over every bucket,
    fused P / Q clears, fused P / Q copies, 1-D segments moved inside the product launches,
    device step counter advanced inside P = M Q) trains like the per-bucket immediate exchange
    and like the CPU reference path (same Q: the Philox draw is host/device identical)."""
    import torch.nn as nn
    import torch.nn.functional as F

    from grace_amd import grace_from_params
    from grace_amd.ops import powersgd as PS
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.comm import LocalComm

    real = PS.randn_shared

    def train(dev, step_level, steps=3):
        torch.manual_seed(0)
        model = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.ReLU(), nn.Conv2d(8, 16, 3, padding=1), nn.ReLU(),
                              nn.AdaptiveAvgPool2d(2), nn.Flatten(), nn.Linear(64, 300), nn.ReLU(),
                              nn.Linear(300, 200), nn.ReLU(), nn.Linear(200, 10)).to(dev)
        grc = grace_from_params({"compressor": "powersgd", "compress_rank": 2, "memory": "powersgd",
                                 "communicator": "allreduce", "world_size": 1}, comm=LocalComm())
        opt = DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.5), grc,
                                   named_parameters=model.named_parameters(), bucket_cap_mb=0.1,
                                   overlap=False, group_collectives=False)
        grc.compressor.enable_step_level(step_level)
        assert len(opt.engine.buckets) >= 3
        for s in range(steps):
            g = torch.Generator().manual_seed(100 * s)
            x, y = torch.randn(4, 3, 8, 8, generator=g).to(dev), torch.randint(0, 10, (4,), generator=g).to(dev)
            opt.zero_grad()
            F.cross_entropy(model(x), y).backward()
            opt.step()
        if dev == "cuda" and step_level:
            assert grc.compressor._arena.get("mtp") is not None  # the merged launch ran
        return [p.detach().cpu() for p in model.parameters()]

    def shared_q(n, seed, device, step=None, zero=None):  # CPU path: the device generator's draw
        if torch.device(device).type == "cpu":
            if zero is not None:
                zero.zero_()
            return real(n, seed, "cuda").cpu()
        return real(n, seed, device, step=step, zero=zero)

    PS.randn_shared = shared_q
    try:
        a = train("cuda", True)
        b = train("cuda", False)
        c = train("cpu", True)
    finally:
        PS.randn_shared = real
    for pa, pb, pc in zip(a, b, c):
        torch.testing.assert_close(pa, pb, rtol=1e-4, atol=1e-5)
        torch.testing.assert_close(pa, pc, rtol=1e-4, atol=1e-5)
