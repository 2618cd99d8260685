"""GPU numerics: BatchNorm(+ReLU) applied inside the consuming convolution's GEMM (operand-loader
prologue, csrc/kernels/gemm_f32.hip BnApplyPro) with the BN backward reduction in the data-grad
epilogue (ReLU test recomputed from x) -- kernels against a plain PyTorch float64 reference, and
the fused ResNet bottleneck (ops/bnconv.py) against the unfused path: outputs, every gradient
and the running statistics."""
import copy

import pytest
import torch
import torch.nn.functional as F

from grace_amd.ops import _native
from grace_amd.ops import bnconv as BC

pytestmark = pytest.mark.gpu


def _cl(t):
    return t.float().cuda().contiguous(memory_format=torch.channels_last)


def _close(got, ref, what, tol=2e-5):
    err = (got.double().cpu() - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-30
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs max |ref| {scale:.3e}"


def _save(C, g):
    mean = torch.randn(C, generator=g) * 0.1
    invstd = torch.rand(C, generator=g) + 0.5
    scale = torch.randn(C, generator=g)
    shift = torch.randn(C, generator=g) * 0.5
    return torch.cat([mean, invstd, scale, shift, torch.zeros(2 * C)]).cuda(), scale.double(), shift.double(), mean


@pytest.mark.parametrize("ksize", [1, 3])
@pytest.mark.parametrize("relu", [True, False])
def test_prologue_forward_and_weight_grad(ksize, relu):
    N, C, H, W, Co = 3, 64, 9, 11, 96
    g = torch.Generator().manual_seed(ksize + 2 * relu)
    x = torch.randn(N, C, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Co, C, ksize, ksize, generator=g, dtype=torch.float64) / (ksize * C ** 0.5)
    dy = torch.randn(N, Co, H, W, generator=g, dtype=torch.float64)
    save, sc, sh, _ = _save(C, g)
    a = x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
    a = a.clamp_min(0) if relu else a
    wr = w.clone().requires_grad_()
    yr = F.conv2d(a, wr, None, 1, (ksize - 1) // 2)
    yr.backward(dy)
    Cn = _native.lib()
    xg, wg, dyg = _cl(x), _cl(w), _cl(dy)
    y = torch.empty(N, Co, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    M = N * H * W
    if ksize == 1:
        Cn.gemm_f32(xg, True, C, wg.reshape(Co, C), True, C, y, Co, M, Co, C, 1, 0, x_save=save, x_relu=relu, x_op=1)
    else:
        Cn.conv3x3_f32(0, xg, wg, y, 1, 1, 0, None, 3, x_save=save, x_relu=relu)
    _close(y, yr.detach(), "fwd")
    if ksize == 1:
        dw = torch.empty(Co, C, device="cuda")
        Cn.gemm_f32(dyg, False, Co, xg, False, C, dw, C, Co, C, M, 0, 0, x_save=save, x_relu=relu, x_op=2)
        _close(dw.view(Co, C, 1, 1), wr.grad, "wgrad")
    else:
        dw = torch.empty(Co, C, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)
        Cn.conv3x3_f32(2, xg, dyg, dw, 1, 0, 0, None, 3, x_save=save, x_relu=relu)
        _close(dw, wr.grad, "wgrad")


@pytest.mark.parametrize("ksize", [1, 3])
def test_epilogue_recomputed_relu(ksize):
    N, C, H, W, Co = 2, 64, 10, 10, 64
    g = torch.Generator().manual_seed(11 + ksize)
    x = torch.randn(N, C, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Co, C, ksize, ksize, generator=g, dtype=torch.float64) / C
    dy = torch.randn(N, Co, H, W, generator=g, dtype=torch.float64)
    save, sc, sh, mean = _save(C, g)
    Cn = _native.lib()
    xg, wg, dyg = _cl(x), _cl(w), _cl(dy)
    da = torch.empty(N, C, H, W, device="cuda").contiguous(memory_format=torch.channels_last)
    M = N * H * W
    part = torch.empty(((M + 63) // 64) * 2 * C, device="cuda")
    if ksize == 1:
        t = Cn.gemm_f32(dyg, True, Co, wg.reshape(Co, C), False, C, da, C, M, C, Co, 1, 0, part, xg, None, save, True)
    else:
        t = Cn.conv3x3_f32(1, dyg, wg, da, 1, 1, 0, part, 3, xg, None, save, True)
    p = part[: t * 2 * C].view(t, 2, C).double().sum(0).cpu()
    xf = x.float().double()  # the kernel tests the fp32 values
    on = (xf * sc.float().double().view(1, -1, 1, 1) + sh.float().double().view(1, -1, 1, 1)) > 0
    dz = da.double().cpu() * on
    torch.testing.assert_close(p[0], dz.sum((0, 2, 3)), rtol=1e-5, atol=1e-4)
    xh = xf - mean.double().view(1, -1, 1, 1)
    torch.testing.assert_close(p[1], (dz * xh).sum((0, 2, 3)), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("stride,cin", [(1, 256), (2, 256), (1, 64)])
def test_fused_bottleneck_matches_unfused(stride, cin, mode):
    from grace_amd.models.resnet import Bottleneck
    from grace_amd.ops.bnact import BatchNormAct2d

    torch.manual_seed(5)
    planes = 64
    down = None
    if stride != 1 or cin != planes * 4:
        from grace_amd.models.resnet import _conv1x1

        down = torch.nn.Sequential(_conv1x1(cin, planes * 4, stride), BatchNormAct2d(planes * 4))
    blk = Bottleneck(cin, planes, stride, down).cuda().to(memory_format=torch.channels_last)
    for m in blk.modules():  # non-trivial affine parameters
        if isinstance(m, BatchNormAct2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    ref = copy.deepcopy(blk)
    x0 = torch.randn(4, cin, 14, 14, device="cuda").contiguous(memory_format=torch.channels_last)

    def run(model, fused):
        BC.set_enabled(fused, mode)
        try:
            x = x0.clone().requires_grad_()
            out = model(x)
            y = out[0] if isinstance(out, tuple) else out
            y.square().mean().backward()
            torch.cuda.synchronize()
            return y.detach(), x.grad, {n: p.grad.clone() for n, p in model.named_parameters()}, \
                {n: b.clone() for n, b in model.named_buffers()}
        finally:
            BC.set_enabled(default[0], default[1])

    default = (BC._ON, BC._MODE)
    calls = {"n": 0}
    real = BC._BnActConvFn.apply

    def counting(*a):
        calls["n"] += 1
        return real(*a)

    BC._BnActConvFn.apply = counting
    try:
        yf, dxf, gf, bf = run(blk, True)
    finally:
        BC._BnActConvFn.apply = real
    assert calls["n"] == (2 if stride == 1 and mode == 1 else 1), calls  # bn1 -> conv2 only in mode 1, stride 1
    yu, dxu, gu, bu = run(ref, False)
    torch.testing.assert_close(yf, yu, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dxf, dxu, rtol=1e-3, atol=1e-6)
    for n in gu:
        torch.testing.assert_close(gf[n], gu[n], rtol=1e-3, atol=1e-5, msg=lambda m, n=n: f"{n}: {m}")
    for n in bu:
        torch.testing.assert_close(bf[n].float(), bu[n].float(), rtol=1e-4, atol=1e-6, msg=lambda m, n=n: f"{n}: {m}")


def test_fused_basic_block_matches_unfused():
    from grace_amd.models.resnet import BasicBlock
    from grace_amd.ops.bnact import BatchNormAct2d

    torch.manual_seed(6)
    blk = BasicBlock(64, 64, 1, None).cuda().to(memory_format=torch.channels_last)
    for m in blk.modules():
        if isinstance(m, BatchNormAct2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    ref = copy.deepcopy(blk)
    x0 = torch.randn(8, 64, 16, 16, device="cuda").contiguous(memory_format=torch.channels_last)
    res = []
    default = (BC._ON, BC._MODE)
    for model, fused in ((blk, True), (ref, False)):
        BC.set_enabled(fused, 1)
        try:
            x = x0.clone().requires_grad_()
            y = model(x)[0]
            y.square().mean().backward()
            torch.cuda.synchronize()
            res.append((y.detach(), x.grad, [p.grad.clone() for p in model.parameters()]))
        finally:
            BC.set_enabled(default[0], default[1])
    (yf, dxf, gf), (yu, dxu, gu) = res
    torch.testing.assert_close(yf, yu, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dxf, dxu, rtol=1e-3, atol=1e-6)
    for a, b in zip(gf, gu):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-5)
