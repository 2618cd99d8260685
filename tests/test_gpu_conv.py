"""GPU: the hand-written f32 MFMA GEMM (csrc/kernels/gemm_f32.hip) and the 1x1 convolution built on
it, against fp64 PyTorch references (exact-f32 MFMA: error ~ 1e-7 of sum |a b| per output)."""
import pytest
import torch
import torch.nn.functional as F

from grace_amd.ops import _native
from grace_amd.ops import conv as conv_mod
from grace_amd.ops.conv import Conv1x1F32, gemm

pytestmark = pytest.mark.gpu


def _operand(rows, k, kc, ld_pad, g):
    """a [rows, k] logical operand stored K-contiguous (rows x ld) or MN-contiguous (k x ld)."""
    logical = torch.randn(rows, k, generator=g, dtype=torch.float64)
    if kc:
        buf = torch.zeros(rows, k + ld_pad, dtype=torch.float64)
        buf[:, :k] = logical
        return logical, buf.float().cuda(), k + ld_pad
    buf = torch.zeros(k, rows + ld_pad, dtype=torch.float64)
    buf[:, :rows] = logical.t()
    return logical, buf.float().cuda(), rows + ld_pad


@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("m,n,k,splits", [(200, 132, 68, 1), (64, 256, 1000, 4), (1568, 64, 512, 1),
                                          (60, 40, 36, 1), (333, 520, 96, 3), (200, 132, 1024, 0),
                                          (1568, 512, 2048, 0)])
def test_gemm_f32_layouts(a_kc, b_kc, m, n, k, splits):
    assert _native.available()
    g = torch.Generator().manual_seed(m * 7 + n)
    if not a_kc and m % 4:
        m += 4 - m % 4
    if not b_kc and n % 4:
        n += 4 - n % 4
    A, a, lda = _operand(m, k, a_kc, 4, g)
    B, b, ldb = _operand(n, k, b_kc, 8, g)
    c = torch.full((m, n), float("nan"), device="cuda")
    gemm(a, a_kc, lda, b, b_kc, ldb, c, n, m, n, k, splits)
    ref = A.float().double() @ B.float().double().t()
    bound = (A.float().double().abs() @ B.float().double().abs().t()) * 2e-6 + 1e-30
    err = (c.double().cpu() - ref).abs()
    assert torch.isfinite(c).all()
    assert (err <= bound).all(), err.max()


@pytest.mark.parametrize("tile", [1, 2, 3, 4])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("m,n,k,splits", [(200, 132, 68, 1), (64, 256, 1000, 4), (333, 520, 96, 3),
                                          (1568, 512, 2048, 0)])
def test_gemm_f32_forced_tiles(tile, a_kc, b_kc, m, n, k, splits):
    """Every forced tile shape: K not a multiple of the 32-k slice, split-K, ragged edges."""
    g = torch.Generator().manual_seed(m * 3 + n + tile)
    if not a_kc and m % 4:
        m += 4 - m % 4
    if not b_kc and n % 4:
        n += 4 - n % 4
    A, a, lda = _operand(m, k, a_kc, 4, g)
    B, b, ldb = _operand(n, k, b_kc, 8, g)
    c = torch.full((m, n), float("nan"), device="cuda")
    gemm(a, a_kc, lda, b, b_kc, ldb, c, n, m, n, k, splits, tile)
    ref = A.float().double() @ B.float().double().t()
    bound = (A.float().double().abs() @ B.float().double().abs().t()) * 2e-6 + 1e-30
    err = (c.double().cpu() - ref).abs()
    assert torch.isfinite(c).all()
    assert (err <= bound).all(), err.max()


def test_gemm_f32_rejects_removed_tile_codes():
    """The 64-k-slice tile codes 5-7 were deleted (round 5): the binding refuses them."""
    a = torch.randn(64, 64, device="cuda")
    c = torch.empty(64, 64, device="cuda")
    for tile in (5, 7, -1):
        with pytest.raises(RuntimeError, match="tile"):
            gemm(a, True, 64, a, True, 64, c, 64, 64, 64, 64, 1, tile)


@pytest.mark.parametrize("nb,cin,cout,hw", [(4, 64, 256, 14), (2, 256, 64, 7), (3, 128, 512, 5), (2, 512, 128, 9)])
def test_conv1x1_f32_fwd_bwd(nb, cin, cout, hw):
    torch.manual_seed(0)
    conv_mod.set_enabled(True)
    conv = Conv1x1F32(cin, cout).cuda()
    x = torch.randn(nb, cin, hw, hw, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = conv(x)
    assert y.is_contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().double().cpu().requires_grad_(True)
    wr = conv.weight.detach().double().cpu().requires_grad_(True)
    yr = F.conv2d(xr, wr)
    yr.backward(dy.double().cpu())
    torch.testing.assert_close(y.detach().double().cpu(), yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad.double().cpu(), xr.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(conv.weight.grad.double().cpu(), wr.grad, rtol=1e-5, atol=1e-4)
    conv_mod.set_enabled(False)


@pytest.mark.parametrize("nb,cin,cout,hw", [(4, 64, 256, 14), (2, 512, 128, 8), (8, 1024, 256, 14)])
def test_conv1x1_autotuned_dispatch(nb, cin, cout, hw):
    """The per-direction autotuned 1x1 path (MIOpen / hipBLASLt / MFMA GEMM, the fastest per
    direction) computes the same convolution as the fp64 reference, and records its choices."""
    torch.manual_seed(1)
    conv_mod.set_enabled(False)
    conv_mod.set_autotune(True)
    conv = Conv1x1F32(cin, cout).cuda()
    x = torch.randn(nb, cin, hw, hw, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_(True)
    for _ in range(2):  # first call tunes, second replays the choice
        x.grad = None
        conv.weight.grad = None
        y = conv(x)
        dy = torch.randn_like(y)
        y.backward(dy)
    assert y.is_contiguous(memory_format=torch.channels_last)
    xr = x.detach().double().cpu().requires_grad_(True)
    wr = conv.weight.detach().double().cpu().requires_grad_(True)
    yr = F.conv2d(xr, wr)
    yr.backward(dy.double().cpu())
    torch.testing.assert_close(y.detach().double().cpu(), yr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad.double().cpu(), xr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(conv.weight.grad.double().cpu(), wr.grad, rtol=1e-4, atol=1e-3)
    m = nb * hw * hw
    got = {d for d, mm, ci, co, _, _ in conv_mod.autotune_table() if (mm, ci, co) == (m, cin, cout)}
    assert got == {"fwd", "dgrad", "wgrad"}


@pytest.mark.parametrize("nb,cin,cout,hw,relu,res", [(4, 64, 256, 14, True, True), (2, 512, 128, 8, True, False),
                                                     (8, 256, 64, 16, False, False)])
def test_conv_bn_stats_epilogue_matches_unfused(nb, cin, cout, hw, relu, res):
    """GEMM with the BN-statistics epilogue + fold + apply == conv + the fused BN's own
    statistics pass: same outputs, running statistics and gradients (fp32)."""
    from grace_amd.ops.bnact import BatchNormAct2d

    torch.manual_seed(2)
    conv_mod.set_enabled(False)
    conv_a = Conv1x1F32(cin, cout).cuda()
    bn_a = BatchNormAct2d(cout, relu=relu).cuda()
    conv_b = Conv1x1F32(cin, cout).cuda()
    bn_b = BatchNormAct2d(cout, relu=relu).cuda()
    conv_b.load_state_dict(conv_a.state_dict())
    with torch.no_grad():
        bn_a.weight.uniform_(0.5, 1.5)
        bn_a.bias.uniform_(-0.2, 0.2)
    bn_b.load_state_dict(bn_a.state_dict())
    x = torch.randn(nb, cin, hw, hw, device="cuda").contiguous(memory_format=torch.channels_last)
    r = torch.randn(nb, cout, hw, hw, device="cuda").contiguous(memory_format=torch.channels_last) if res else None
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    key = (nb * hw * hw, cin, cout, relu, res)
    conv_mod._BN_CHOICE[key] = "stats_t2"  # force the fused path for this shape
    ya = conv_mod.conv_bn_act(conv_a, bn_a, xa, r)
    yb = bn_b(conv_b(xb), r)
    dy = torch.randn_like(ya)
    ya.backward(dy)
    yb.backward(dy)
    torch.testing.assert_close(ya, yb, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(bn_a.running_mean, bn_b.running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(bn_a.running_var, bn_b.running_var, rtol=1e-4, atol=1e-5)
    assert int(bn_a.num_batches_tracked) == int(bn_b.num_batches_tracked) == 1
    torch.testing.assert_close(xa.grad, xb.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(conv_a.weight.grad, conv_b.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(bn_a.weight.grad, bn_b.weight.grad, rtol=1e-4, atol=1e-3)
    del conv_mod._BN_CHOICE[key]
