"""Single-process (W=1) semantics of every compressor against the golden oracles (CPU)."""
import math

import pytest
import torch

import os
import sys
sys.path.insert(0, os.path.dirname(__file__))
import oracles as O  # noqa: E402
from grace_amd import compressor as Z
from grace_amd import memory as M
from grace_amd.communicator import Allgather, Allreduce, Broadcast
from grace_amd.core import register_layout
from grace_amd.ops.layout import SegmentLayout
from grace_amd.parallel.comm import LocalComm


def _x(*shape, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g)


def roundtrip(comp, x, name="t"):
    payload, ctx = comp.compress(x, name)
    return comp.decompress(payload, ctx)


def test_none_fp16():
    x = _x(100)
    assert torch.equal(roundtrip(Z.NoneCompressor(), x), x)
    torch.testing.assert_close(roundtrip(Z.FP16Compressor(), x), O.fp16(x))
    bf = roundtrip(Z.FP16Compressor(torch.bfloat16), x)
    torch.testing.assert_close(bf, x.bfloat16().float())


@pytest.mark.parametrize("shape", [(1,), (3,), (64,), (1000,), (17, 33), (8, 3, 3, 3)])
@pytest.mark.parametrize("ratio", [0.01, 0.3])
def test_topk_matches_oracle(shape, ratio):
    x = _x(*shape)
    torch.testing.assert_close(roundtrip(Z.TopKCompressor(ratio), x), O.topk(x, ratio))


def test_threshold_matches_oracle():
    x = _x(5000) * 0.02
    torch.testing.assert_close(roundtrip(Z.ThresholdCompressor(0.01), x), O.threshold(x, 0.01))


def test_sign_family_single_rank():
    x = _x(777)
    torch.testing.assert_close(roundtrip(Z.SignSGDCompressor(), x), torch.where(x >= 0, 1.0, -1.0))
    torch.testing.assert_close(roundtrip(Z.EFSignSGDCompressor(0.1), x), O.efsign(x), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(roundtrip(Z.OneBitCompressor(), x), O.onebit(x), rtol=1e-5, atol=1e-6)


def test_signum_momentum():
    c = Z.SignumCompressor(0.9)
    x1, x2 = _x(300, seed=1), _x(300, seed=2)
    roundtrip(c, x1, "p")
    out = roundtrip(c, x2, "p")
    m = 0.1 * x2 + 0.9 * x1
    torch.testing.assert_close(out, torch.where(m >= 0, 1.0, -1.0))


def test_qsgd_error_bound_and_unbiased():
    x = _x(4000)
    c = Z.QSGDCompressor(64)
    dec = roundtrip(c, x)
    assert (dec - x).abs().max() <= O.qsgd_bounds(x, 64) * (1 + 1e-5)
    acc = torch.zeros_like(x)
    n = 200
    for i in range(n):
        acc += roundtrip(c, x, "q")
    err = (acc / n - x).abs().mean() / x.abs().mean()
    assert err < 0.05


def test_terngrad_values_and_unbiased_within_clip():
    x = _x(3000)
    c = Z.TernGradCompressor()
    dec = roundtrip(c, x)
    scal = O.terngrad_scalar(x)
    vals = set(torch.unique(dec / scal).round().tolist())
    assert vals <= {-1.0, 0.0, 1.0}
    acc = torch.zeros_like(x)
    for _ in range(300):
        acc += roundtrip(c, x, "t")
    clipped = torch.clamp(x, -scal, scal)
    assert ((acc / 300 - clipped).abs().mean() / clipped.abs().mean()) < 0.08


def test_natural_power_of_two_and_unbiased():
    x = _x(2000)
    c = Z.NaturalCompressor()
    dec = roundtrip(c, x)
    lo, hi = O.natural_decode_range(x)
    a = dec.abs()
    assert torch.all((torch.isclose(a, lo) | torch.isclose(a, hi)))
    assert torch.all(torch.sign(dec) == torch.sign(x))
    acc = torch.zeros_like(x)
    for _ in range(200):
        acc += roundtrip(c, x, "n")
    assert ((acc / 200 - x).abs().mean() / x.abs().mean()) < 0.05


def test_u8bit_close():
    x = _x(1000)
    dec = roundtrip(Z.U8bitCompressor(), x)
    assert (dec - x).abs().max() <= 0.05 * x.abs().max()


def test_sketch_bins():
    x = _x(5000)
    dec = roundtrip(Z.SketchCompressor(64), x)
    assert torch.unique(dec).numel() <= 64
    assert (dec - x).abs().mean() < 0.1


def test_inceptionn_classes():
    x = torch.tensor([2.0, -3.5, 0.75, -0.3, 1e-3, 1e-12, 0.0])
    dec = roundtrip(Z.INCEPTIONNCompressor(2e-10), x)
    assert dec[0] == 2.0 and dec[1] == -3.5  # fp32 class exact
    assert abs(dec[2] - 0.75) < 1e-3 and abs(dec[3] + 0.3) < 1e-3  # 16-bit class
    assert dec[5] == 0 and dec[6] == 0  # dropped


def test_adaq_means():
    x = _x(10000)
    c = Z.AdaqCompressor(0.05)
    dec = roundtrip(c, x)
    vals = torch.unique(dec)
    assert vals.numel() <= 3  # {minus_mean, 0, plus_mean}
    assert 0.02 * x.numel() < (dec != 0).sum() < 0.2 * x.numel()


def test_dgc_selects_about_ratio():
    x = _x(20000)
    c = Z.DgcCompressor(0.01)
    payload, ctx = c.compress(x, "d")
    hdr = payload[0]
    n = int(hdr[0])
    assert 0.5 * 200 <= n <= 1.5 * 200
    assert payload[1].numel() == 400  # capacity 2 x target: fixed payload size
    dec = c.decompress(payload, ctx)
    sel = dec != 0
    assert sel.sum() == n
    assert torch.equal(dec[sel], x[sel])


def test_capacity_payload_fixed_size_and_spill():
    """Threshold with capacity < selected: the payload size is fixed, the header holds the
    selected count, and the spilled entries stay in the residual (error feedback keeps them)."""
    from grace_amd.ops import cappayload as P

    x = _x(5000)
    full = Z.ThresholdCompressor(0.5)
    p_full, _ = full.compress(x, "t")
    n_sel = int((x.abs() > 0.5).sum())
    assert int(p_full[0][0]) == n_sel and p_full[1].numel() == 5000
    c = Z.ThresholdCompressor(0.5, capacity=0.05)
    mem = M.ResidualMemory()
    grc = Allgather(c, mem, comm=LocalComm())
    out = grc.step(x.clone(), "t")
    cap = P.capacity(5000, 0.05)
    assert (out != 0).sum() == cap < n_sel
    r = mem.residuals["t"]
    # sent + residual == input; residual still holds the spilled large entries
    torch.testing.assert_close(out + r, x)
    assert int((r.abs() > 0.5).sum()) == n_sel - cap


def test_powersgd_matches_oracle_w1():
    m = _x(40, 30)
    c = Z.PowerSGDCompressor(rank=3)
    grc = Allreduce(c, M.NoneMemory(), comm=LocalComm())
    out = grc.step(m, "w")
    # oracle with the same initial Q
    from grace_amd.ops import powersgd as PS
    from grace_amd.ops.randomk import fnv1a64

    plan = PS.plan_for(SegmentLayout((1200,), ((40, 30),)), 3)
    seed = (fnv1a64(b"w") ^ 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    q0 = PS.randn_shared(plan.q_total, seed, "cpu").view(30, 3)
    q0 = O.gram_schmidt(q0)
    torch.testing.assert_close(out, O.powersgd(m, q0), rtol=1e-4, atol=1e-5)


def test_powersgd_vector_passthrough():
    v = _x(50)
    c = Z.PowerSGDCompressor(rank=2)
    grc = Allreduce(c, M.NoneMemory(), comm=LocalComm())
    torch.testing.assert_close(grc.step(v, "b"), v)


# ------------------------------------------------------------------ bucket == per tensor
@pytest.mark.parametrize("make", [
    lambda: Z.TopKCompressor(0.05),
    lambda: Z.SignSGDCompressor(),
    lambda: Z.EFSignSGDCompressor(0.1),
    lambda: Z.OneBitCompressor(),
    lambda: Z.U8bitCompressor(),
])
def test_bucket_equals_per_tensor(make):
    shapes = [(10, 7), (64,), (3, 3, 3, 3), (1,), (129,)]
    ts = [_x(*s, seed=i) for i, s in enumerate(shapes)]
    flat = torch.cat([t.flatten() for t in ts])
    lay = SegmentLayout.from_tensors(ts)
    register_layout("bucket0", lay)
    c = make()
    got = roundtrip(c, flat, "bucket0")
    exp = torch.cat([roundtrip(make(), t, f"t{i}").flatten() for i, t in enumerate(ts)])
    torch.testing.assert_close(got, exp, rtol=1e-5, atol=1e-6)


# ------------------------------------------------------------------ memories
def test_residual_fused_equals_generic():
    x1, x2 = _x(500, seed=3), _x(500, seed=4)
    fused = Allgather(Z.TopKCompressor(0.1), M.ResidualMemory(), comm=LocalComm())
    out1 = [fused.step(x, "w") for x in (x1, x2)]

    class Plain(Z.TopKCompressor):
        def fused_compress(self, *a):
            return None

    plain = Allgather(Plain(0.1), M.ResidualMemory(), comm=LocalComm())
    out2 = [plain.step(x, "w") for x in (x1, x2)]
    for a, b in zip(out1, out2):
        torch.testing.assert_close(a, b)
    torch.testing.assert_close(fused.memory.residuals["w"], plain.memory.residuals["w"])


def test_error_feedback_conserves_mass():
    """sum over steps of sent + final residual == sum of gradients (EF invariant)."""
    grc = Allgather(Z.TopKCompressor(0.02), M.ResidualMemory(), comm=LocalComm())
    total_g = torch.zeros(1000)
    total_sent = torch.zeros(1000)
    for s in range(5):
        g = _x(1000, seed=10 + s)
        total_g += g
        total_sent += grc.step(g, "w")
    torch.testing.assert_close(total_sent + grc.memory.residuals["w"], total_g, rtol=1e-5, atol=1e-5)


def test_dgc_memory_momentum_and_masking():
    mem = M.DgcMemory(momentum=0.9, gradient_clipping=False)
    grc = Allgather(Z.DgcCompressor(0.05), mem, comm=LocalComm())
    g = _x(4000)
    out = grc.step(g, "w")
    sent = out != 0
    assert torch.all(mem.residuals["w"][sent] == 0) and torch.all(mem.gradients["w"][sent] == 0)
    assert torch.equal(mem.gradients["w"][~sent], g[~sent])


def test_dgc_memory_clipping_runs():
    mem = M.DgcMemory(momentum=0.9, gradient_clipping=True)
    grc = Allgather(Z.DgcCompressor(0.05), mem, comm=LocalComm())
    g = _x(1000)
    out = grc.step(g, "w")
    assert torch.isfinite(out).all()
    assert out.abs().max() <= g.norm() + 1e-5


def test_powersgd_memory_residual():
    mem = M.PowerSGDMemory(compress_rank=2)
    c = Z.PowerSGDCompressor(rank=2)
    grc = Allreduce(c, mem, comm=LocalComm())
    m = _x(20, 10)
    out = grc.step(m, "w")
    torch.testing.assert_close(mem.residuals["w"], m - out, rtol=1e-5, atol=1e-5)


def test_state_dict_roundtrip():
    grc = Allgather(Z.SignumCompressor(0.9), M.ResidualMemory(), comm=LocalComm())
    grc.step(_x(100), "a")
    sd = grc.state_dict()
    grc2 = Allgather(Z.SignumCompressor(0.9), M.ResidualMemory(), comm=LocalComm())
    grc2.load_state_dict(sd)
    x = _x(100, seed=5)
    torch.testing.assert_close(grc.step(x, "a"), grc2.step(x, "a"))


def test_broadcast_single_rank():
    grc = Broadcast(Z.TopKCompressor(0.1), M.NoneMemory(), comm=LocalComm())
    x = _x(300)
    torch.testing.assert_close(grc.step(x, "x"), O.topk(x, 0.1))


def test_allreduce_rejects_nonlinear():
    with pytest.raises(ValueError):
        Allreduce(Z.TopKCompressor(0.1), M.NoneMemory(), comm=LocalComm())


def test_powersgd_fused_memory_matches_unfused():
    """fused_compress (compensate inside M Q, residual inside P Q^T) == the generic
    compensate -> compress -> update sequence, over 3 steps of a bucket with 1-D segments."""
    from grace_amd.core import register_layout
    from grace_amd.ops.layout import SegmentLayout

    class Unfused(M.PowerSGDMemory):
        pass

    shapes = [(20, 10), (7,), (6, 3, 2, 2), (5,)]
    register_layout("psgd_bucket", SegmentLayout.from_tensors([torch.empty(s) for s in shapes]))
    outs = {}
    for mem_cls in (M.PowerSGDMemory, Unfused):
        mem = mem_cls(compress_rank=2)
        grc = Allreduce(Z.PowerSGDCompressor(rank=2), mem, comm=LocalComm())
        res = []
        for s in range(3):
            g = torch.cat([_x(*sh, seed=10 * s + i).flatten() for i, sh in enumerate(shapes)])
            res.append(grc.step(g, "psgd_bucket").clone())
        res.append(mem.residuals["psgd_bucket"].clone())
        outs[mem_cls] = res
    for a, b in zip(outs[M.PowerSGDMemory], outs[Unfused]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


def test_qsgd_code_dtypes_are_reducible():
    """Shared-scale (all-reduced) codes never use int16: RCCL and gloo have no int16 reduction."""
    from grace_amd.compressor.qsgd import QSGDCompressor

    c = QSGDCompressor(127)
    assert c.code_dtype(1) == torch.int8
    assert c.code_dtype(4) == torch.int8 and QSGDCompressor(255).code_dtype(4) == torch.int16  # gathered: no reduction
    c.enable_allreduce_mode()
    assert c.code_dtype(1) == torch.int8
    assert c.code_dtype(2) == torch.float16 and c.code_dtype(8) == torch.float16  # 1016 <= 2048: exact
    assert c.code_dtype(32) == torch.int32
    assert QSGDCompressor(15, shared_scale=True).code_dtype(8) == torch.int8


@pytest.mark.parametrize("s,bits", [(1, 2), (3, 4), (7, 4)])
def test_qsgd_small_s_codes_are_bit_packed(s, bits):
    """s = 1 -> 2-bit, s <= 7 -> 4-bit codes on the wire; decoding the packed payload gives
    exactly the int8-code result (same rounding stream)."""
    class Unpacked(Z.QSGDCompressor):
        @property
        def pack_bits(self):
            return 0

    x = _x(4001)
    cp, cu = Z.QSGDCompressor(s), Unpacked(s)
    tp, ctxp = cp.compress(x, "w")
    tu, ctxu = cu.compress(x, "w")
    assert tp[0].dtype == torch.uint8 and tp[0].numel() == (x.numel() * bits + 7) // 8
    assert tu[0].dtype == torch.int8
    torch.testing.assert_close(cp.decompress(tp, ctxp), cu.decompress(tu, ctxu), rtol=0, atol=0)
