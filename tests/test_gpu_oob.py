"""GPU: out-of-bounds / input-clobber canaries for the hand-written GEMM and conv kernels.

Every output is placed as a view inside a larger buffer pre-filled with a canary bit pattern and
every input is checked unchanged afterwards: a kernel that writes outside its output (a tile edge,
the split-K zero fill, the statistics epilogue) or into an operand fails here with the offending
byte range, instead of corrupting whatever tensor the caching allocator put next to it.
Shapes: resnet18_cifar at batch 8 (the plain-DDP test's model) and the small ResNet-50 layers."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CANARY = -1.2345e-31  # a bit pattern no kernel produces from these inputs
GUARD = 4096  # floats on each side


def _lib():
    from grace_amd.ops import _native

    return _native.lib()


def _guarded_cl(n, c, h, w):
    """(buffer, channels_last (n, c, h, w) view inside it)"""
    numel = n * c * h * w
    buf = torch.full((numel + 2 * GUARD,), CANARY, device="cuda")
    view = buf[GUARD:GUARD + numel].view(n, h, w, c).permute(0, 3, 1, 2)
    assert view.is_contiguous(memory_format=torch.channels_last)
    return buf, view


def _guarded_flat(numel):
    buf = torch.full((numel + 2 * GUARD,), CANARY, device="cuda")
    return buf, buf[GUARD:GUARD + numel]


def _check_guards(buf, numel, what):
    lo, hi = buf[:GUARD], buf[GUARD + numel:]
    bad_lo = (lo != CANARY).nonzero()
    bad_hi = (hi != CANARY).nonzero()
    assert bad_lo.numel() == 0, f"{what}: {bad_lo.numel()} floats written BEFORE the output (first at -{GUARD - int(bad_lo[0])})"
    assert bad_hi.numel() == 0, f"{what}: {bad_hi.numel()} floats written AFTER the output (first at +{int(bad_hi[0])})"


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


# (N, Cin, H, W, Cout, stride, ksize)
SHAPES = [
    (8, 64, 16, 16, 64, 1, 3), (8, 64, 16, 16, 128, 2, 3), (8, 64, 16, 16, 128, 2, 1),
    (8, 128, 8, 8, 128, 1, 3), (8, 128, 8, 8, 256, 2, 3), (8, 128, 8, 8, 256, 2, 1),
    (8, 256, 4, 4, 256, 1, 3), (8, 256, 4, 4, 512, 2, 3), (8, 256, 4, 4, 512, 2, 1),
    (8, 512, 2, 2, 512, 1, 3),
    (32, 256, 14, 14, 256, 1, 3), (32, 512, 7, 7, 512, 1, 3), (32, 128, 28, 28, 128, 1, 3),
]


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_conv3x3_no_oob_writes(shape):
    n, cin, h, w, cout, s, k = shape
    ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
    g = torch.Generator(device="cuda").manual_seed(1)
    x = _cl(torch.randn(n, cin, h, w, device="cuda", generator=g))
    wt = _cl(torch.randn(cout, cin, k, k, device="cuda", generator=g) * 0.05)
    dy = _cl(torch.randn(n, cout, ho, wo, device="cuda", generator=g))
    x0, w0, dy0 = x.clone(), wt.clone(), dy.clone()
    C = _lib()
    m_out = n * ho * wo
    for tile in range(0, 5):
        # forward, with and without the statistics epilogue
        for stats in (False, True):
            buf, y = _guarded_cl(n, cout, ho, wo)
            pn = ((m_out + 63) // 64) * 2 * cout
            pbuf, part = _guarded_flat(pn)
            C.conv3x3_f32(0, x, wt, y, s, 1, tile, part if stats else None, k)
            torch.cuda.synchronize()
            _check_guards(buf, y.numel(), f"fwd tile {tile} stats {stats}")
            _check_guards(pbuf, pn, f"fwd stats partials tile {tile}")
            ref = torch.nn.functional.conv2d(x, wt, None, s, (k - 1) // 2)
            torch.testing.assert_close(y, ref, rtol=1e-4, atol=1e-3)
        # weight gradient (split-K auto: zero fill + atomics)
        buf, dw = _guarded_cl(cout, cin, k, k)
        C.conv3x3_f32(2, x, dy, dw, s, 0, tile, None, k)
        torch.cuda.synchronize()
        _check_guards(buf, dw.numel(), f"wgrad tile {tile}")
        # split-K forward (f32 atomics into a zeroed output: the autotuner's mfma_tN_sK)
        for splits in (2, 4):
            buf, y = _guarded_cl(n, cout, ho, wo)
            C.conv3x3_f32(0, x, wt, y, s, splits, tile, None, k)
            torch.cuda.synchronize()
            _check_guards(buf, y.numel(), f"fwd tile {tile} splits {splits}")
            torch.testing.assert_close(y, torch.nn.functional.conv2d(x, wt, None, s, (k - 1) // 2), rtol=1e-4, atol=1e-3)
        # data gradient (3x3 stride 1 only), whole-K and split-K
        if s == 1 and k == 3:
            ref = torch.nn.grad.conv2d_input((n, cin, h, w), wt, dy, padding=1)
            for splits in (1, 2, 4):
                buf, dx = _guarded_cl(n, cin, h, w)
                C.conv3x3_f32(1, dy, wt, dx, 1, splits, tile)
                torch.cuda.synchronize()
                _check_guards(buf, dx.numel(), f"dgrad tile {tile} splits {splits}")
                torch.testing.assert_close(dx, ref, rtol=1e-4, atol=1e-3)
    assert torch.equal(x, x0) and torch.equal(wt, w0) and torch.equal(dy, dy0), "an input operand was written"


@pytest.mark.parametrize("mnk", [(128, 256, 128), (32, 512, 256), (1568, 2048, 512), (100, 36, 68), (3136, 64, 256)])
def test_gemm_f32_no_oob_writes(mnk):
    m, n, k = mnk
    g = torch.Generator(device="cuda").manual_seed(2)
    a = torch.randn(m, k, device="cuda", generator=g)
    b = torch.randn(n, k, device="cuda", generator=g)
    a0, b0 = a.clone(), b.clone()
    C = _lib()
    for tile in range(0, 5):
        for splits in (1, 0, 3):
            buf, c = _guarded_flat(m * n)
            C.gemm_f32(a, True, k, b, True, k, c, n, m, n, k, splits, tile, None, None, None, None, False, None, False, 1)
            torch.cuda.synchronize()
            _check_guards(buf, m * n, f"gemm tile {tile} splits {splits}")
            torch.testing.assert_close(c.view(m, n), a @ b.t(), rtol=1e-4, atol=1e-3)
    assert torch.equal(a, a0) and torch.equal(b, b0)
