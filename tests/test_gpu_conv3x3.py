"""GPU numerics: 3x3 / pad 1 convolutions as implicit GEMMs on the f32 MFMA kernel
(csrc/kernels/gemm_f32.hip modes 2-4) against a plain PyTorch float64 CPU reference, per
direction and tile shape, strides 1 and 2, odd image sizes; and the autotuned module path
(Conv2dSplitGrad -> ops/conv.py _Conv3x3Fn) against nn.Conv2d."""
import pytest
import torch
import torch.nn.functional as F

from grace_amd.ops import _native
from grace_amd.ops import conv as CV

pytestmark = pytest.mark.gpu

SHAPES = [  # (N, Cin, H, W, Cout, stride)
    (2, 32, 7, 7, 64, 1),
    (3, 64, 10, 9, 32, 1),
    (1, 96, 5, 13, 128, 1),
    (2, 64, 12, 12, 128, 2),
    (2, 32, 9, 11, 64, 2),
    (4, 128, 14, 14, 128, 1),
]


def _data(N, Cin, H, W, Cout, s, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, Cin, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / (3 * Cin ** 0.5)
    Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
    dy = torch.randn(N, Cout, Ho, Wo, generator=g, dtype=torch.float64)
    return x, w, dy


def _cl(t):
    return t.float().cuda().contiguous(memory_format=torch.channels_last)


def _close(got, ref, what):
    err = (got.double().cpu() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-30
    assert err <= 2e-5 * scale, f"{what}: max err {err:.3e} vs max |ref| {scale:.3e}"


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4])
def test_conv3x3_implicit_gemm_directions(shape, tile):
    N, Cin, H, W, Cout, s = shape
    x, w, dy = _data(*shape, seed=tile)
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = F.conv2d(xr, wr, None, s, 1)
    yr.backward(dy)
    C = _native.lib()
    xg, wg, dyg = _cl(x), _cl(w), _cl(dy)
    y = torch.empty(yr.shape, device="cuda").contiguous(memory_format=torch.channels_last)
    C.conv3x3_f32(0, xg, wg, y, s, 1, tile)
    _close(y, yr.detach(), "fwd")
    dw = torch.full(w.shape, 3.0, device="cuda").contiguous(memory_format=torch.channels_last)
    C.conv3x3_f32(2, xg, dyg, dw, s, 0, tile)  # split-K zeroes its output itself
    _close(dw, wr.grad, "wgrad")
    if s == 1:
        dx = torch.empty(x.shape, device="cuda").contiguous(memory_format=torch.channels_last)
        C.conv3x3_f32(1, dyg, wg, dx, 1, 1, tile)
        _close(dx, xr.grad, "dgrad")
    torch.cuda.synchronize()


def test_conv3x3_fwd_statistics_epilogue():
    N, Cin, H, W, Cout, s = 4, 64, 14, 14, 96, 1
    x, w, _ = _data(N, Cin, H, W, Cout, s, seed=5)
    C = _native.lib()
    y = torch.empty(N, Cout, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    M = N * H * W
    part = torch.empty(((M + 63) // 64) * 2 * Cout, device="cuda")
    tiles = C.conv3x3_f32(0, _cl(x), _cl(w), y, s, 1, 4, part)
    p = part[: tiles * 2 * Cout].view(tiles, 2, Cout).double().sum(0).cpu()
    yd = y.double().cpu().permute(0, 2, 3, 1).reshape(-1, Cout)
    torch.testing.assert_close(p[0], yd.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(p[1], (yd * yd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("stride", [1, 2])
def test_conv3x3_module_autotuned_matches_conv2d(stride):
    from grace_amd.ops.wgrad import Conv2dSplitGrad

    torch.manual_seed(0)
    m = Conv2dSplitGrad(64, 128, 3, stride=stride, padding=1, bias=False).cuda().to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(64, 128, 3, stride=stride, padding=1, bias=False).double()
    ref.weight.data.copy_(m.weight.detach().double().cpu())
    x = torch.randn(4, 64, 16, 16, dtype=torch.float64)
    xg = _cl(x).requires_grad_()
    xr = x.clone().requires_grad_()
    for _ in range(2):  # the first call autotunes, the second runs the choice
        m.weight.grad = None
        xg.grad = None
        y = m(xg)
        y.backward(torch.ones_like(y))
    yr = ref(xr)
    yr.backward(torch.ones_like(yr))
    torch.cuda.synchronize()
    _close(y.detach(), yr.detach(), "fwd")
    _close(xg.grad, xr.grad, "dgrad")
    _close(m.weight.grad, ref.weight.grad, "wgrad")
    table = CV.conv3x3_autotune_table()
    assert any(r[0] == "fwd" and r[4] == 64 and r[5] == 128 and r[6] == stride for r in table), table


def test_conv3x3_rejects_bad_shapes():
    C = _native.lib()
    x = torch.randn(2, 48, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)  # Cin % 32 != 0
    w = torch.randn(64, 48, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.empty(2, 64, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    with pytest.raises(RuntimeError):
        C.conv3x3_f32(0, x, w, y, 1, 1, 0)
    x2 = torch.randn(2, 64, 8, 8, device="cuda")  # NCHW memory
    w2 = torch.randn(64, 64, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
    with pytest.raises(RuntimeError):
        C.conv3x3_f32(0, x2, w2, y, 1, 1, 0)
