"""NHWC max pooling with 1-byte window codes (csrc/kernels/pool.hip) vs F.max_pool2d in fp32:
outputs bit-identical (max is exact), input gradients equal (ties: first maximum wins, as
PyTorch), including padded windows, overlapping windows (3x3 / 2) and repeated values."""
import pytest
import torch
import torch.nn.functional as F

from grace_amd.ops.pool import MaxPool2dNHWC

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("k,s,p,shape", [
    (3, 2, 1, (4, 64, 56, 56)),    # ResNet stem (scaled down)
    (3, 2, 1, (2, 16, 7, 9)),      # odd sizes, padded edges
    (2, 2, 0, (4, 128, 28, 28)),   # VGG
    (2, 2, 0, (2, 64, 5, 7)),      # odd -> floor
    (3, 1, 1, (2, 32, 6, 6)),      # stride 1: every input in 9 windows
])
@pytest.mark.parametrize("ties", [False, True])
def test_maxpool_matches_torch(k, s, p, shape, dtype, ties):
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(shape, generator=g)
    if ties:
        x = torch.round(x * 2) / 2  # many equal values: exercises the first-maximum rule
    x = x.to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    pool = MaxPool2dNHWC(k, s, p)
    assert pool._native_ok(x)
    xa = x.clone().requires_grad_(True)
    xb = x.clone().float().requires_grad_(True)
    ya = pool(xa)
    yb = F.max_pool2d(xb, k, s, p)
    assert ya.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(ya.float(), yb)
    dy = torch.randn(yb.shape, generator=g).to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    ya.backward(dy)
    yb.backward(dy.float())
    tol = dict(rtol=1e-6, atol=1e-6) if dtype == torch.float32 else dict(rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(xa.grad.float(), xb.grad, **tol)


def test_maxpool_nan_propagates():
    """A NaN wins its window (value and gradient), as in PyTorch.  (All -inf windows are not
    compared: PyTorch's NHWC kernel routes their gradient to element (0, 0) of the image.)"""
    g = torch.Generator(device="cpu").manual_seed(2)
    x = torch.randn(1, 8, 4, 4, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    x[0, 3, 1, 2] = float("nan")
    pool = MaxPool2dNHWC(2, 2)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = pool(xa), F.max_pool2d(xb, 2, 2)
    assert torch.equal(torch.nan_to_num(ya, nan=7.0), torch.nan_to_num(yb, nan=7.0))
    ya.sum().backward()
    yb.sum().backward()
    assert torch.equal(xa.grad, xb.grad)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_global_avgpool_flat_matches_torch(dtype):
    from grace_amd.ops.pool import GlobalAvgPoolFlat

    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(4, 256, 7, 7, generator=g).to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    xa, xb = x.clone().requires_grad_(True), x.clone().float().requires_grad_(True)
    ya = GlobalAvgPoolFlat()(xa)
    yb = torch.flatten(F.adaptive_avg_pool2d(xb, 1), 1)
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(ya.float(), yb, **tol)
    dy = torch.randn(yb.shape, generator=g).to(DEV)
    ya.backward(dy.to(ya.dtype))
    yb.backward(dy)
    assert xa.grad.dtype == dtype and xa.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(xa.grad.float(), xb.grad, **tol)
