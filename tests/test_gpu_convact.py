"""Fused conv bias (+ReLU) kernels (csrc/kernels/bnact.hip bias_act_*) vs the plain PyTorch fp32
ops: y = relu(x + b), dz = dy * [y > 0], dbias = sum over N, H, W of dz."""
import pytest
import torch
import torch.nn.functional as F

from grace_amd.ops.convact import ConvBiasAct2d, bias_act, _fusable

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("relu", [True, False])
@pytest.mark.parametrize("shape", [(4, 64, 56, 56), (8, 512, 14, 14), (2, 128, 7, 9), (3, 1024, 5, 5)])
def test_bias_act_matches_fp32_reference(shape, relu, dtype):
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(shape, generator=g).to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    b = (torch.randn(shape[1], generator=g) * 0.5).to(DEV).requires_grad_(True)
    dy = torch.randn(shape, generator=g).to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    assert _fusable(x)
    xg = x.clone().requires_grad_(True)
    y = bias_act(xg, b, relu)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = xr + br.view(1, -1, 1, 1)
    yr = F.relu(yr) if relu else yr
    yr.backward(dy.float())
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(xg.grad.float(), xr.grad.float() if dtype == torch.float32 else
                               (dy.float() * (yr > 0) if relu else dy.float()), **tol)
    m = x.numel() // shape[1]
    torch.testing.assert_close(b.grad, br.grad, rtol=1e-4, atol=1e-4 * m ** 0.5 if dtype == torch.float32 else 2e-2 * m ** 0.5)


def test_conv_bias_act_module_matches_conv_relu():
    torch.manual_seed(0)
    m = ConvBiasAct2d(32, 64, 3, padding=1).to(DEV).to(memory_format=torch.channels_last)
    ref = torch.nn.Conv2d(32, 64, 3, padding=1).to(DEV).to(memory_format=torch.channels_last)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(4, 32, 20, 20, device=DEV).contiguous(memory_format=torch.channels_last)
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    y = m(x1)
    yr = F.relu(ref(x2))
    torch.testing.assert_close(y, yr, rtol=1e-5, atol=1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    yr.backward(dy)
    torch.testing.assert_close(x1.grad, x2.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(m.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-3)


def test_vgg16_graph_step_runs():
    from grace_amd.models.vgg import vgg16

    torch.manual_seed(0)
    net = vgg16(10).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(2, 3, 64, 64, device=DEV).contiguous(memory_format=torch.channels_last)
    loss = F.cross_entropy(net(x), torch.tensor([1, 2], device=DEV))
    loss.backward()
    assert torch.isfinite(loss) and all(torch.isfinite(p.grad).all() for p in net.parameters())
