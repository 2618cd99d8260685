"""GPU: weight gradients on the side stream (grace_amd/ops/wgrad.py) give the same gradients as the
in-line backward -- eagerly, through the GRACE engine's bucket gather, and inside a captured
whole-step HIP graph (the fork is a parallel graph branch)."""
import pytest
import torch
import torch.nn.functional as F

from grace_amd.ops import wgrad
from grace_amd.ops.wgrad import Conv2dSplitGrad

pytestmark = pytest.mark.gpu


def _grads(model, x, y):
    for p in model.parameters():
        p.grad = None
    loss = F.cross_entropy(model(x), y)
    loss.backward()
    return [p.grad.detach().clone() for p in model.parameters()]


@pytest.mark.parametrize("stride,pad,k", [(1, 1, 3), (2, 1, 3), (2, 0, 1), (2, 3, 7)])
def test_split_conv_matches_conv2d(stride, pad, k):
    torch.manual_seed(0)
    conv = Conv2dSplitGrad(16, 32, k, stride=stride, padding=pad, bias=False).cuda()
    ref = torch.nn.Conv2d(16, 32, k, stride=stride, padding=pad, bias=False).cuda()
    ref.load_state_dict(conv.state_dict())
    x = torch.randn(4, 16, 20, 20, device="cuda").contiguous(memory_format=torch.channels_last)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = conv(xa), ref(xb)
    dy = torch.randn_like(ya)
    ya.backward(dy)
    yb.backward(dy)
    torch.testing.assert_close(ya, yb, rtol=0, atol=0)
    torch.testing.assert_close(xa.grad, xb.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(conv.weight.grad, ref.weight.grad, rtol=1e-5, atol=1e-5)


def test_resnet_side_stream_grads_equal_inline():
    from grace_amd.models import resnet50

    torch.manual_seed(0)
    model = resnet50().cuda().to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (4,), device="cuda")
    wgrad.set_enabled(False)
    try:
        _grads(model, x, y)  # settle autotuned choices (same backend both runs)
        ref = _grads(model, x, y)
    finally:
        wgrad.set_enabled(True)
    got = _grads(model, x, y)
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


def test_engine_graph_with_side_stream_wgrad():
    """Top-K 1 % engine step captured in a whole-step graph with the wgrad fork: replays match
    an eager run step for step (parameters after 3 steps)."""
    from grace_amd import grace_from_params
    from grace_amd.models import resnet50
    from grace_amd.parallel import DistributedOptimizer, FusedSGD
    from grace_amd.parallel.graph import GraphedStep

    def build():
        torch.manual_seed(1)
        m = resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last)
        grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.01, "memory": "residual",
                                 "communicator": "allgather", "world_size": 1})
        opt = DistributedOptimizer(FusedSGD(list(m.parameters()), lr=0.01, momentum=0.5), grc,
                                   named_parameters=list(m.named_parameters()), overlap=False)
        return m, opt

    x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), device="cuda")

    def make_step(m, opt):
        def step():
            opt.zero_grad(set_to_none=True)
            loss = F.cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            return loss
        return step

    m1, o1 = build()
    s1 = make_step(m1, o1)
    for _ in range(6):
        s1()
    m2, o2 = build()
    g = GraphedStep(make_step(m2, o2), warmup=3)
    for _ in range(3):
        g()
    torch.cuda.synchronize()
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5, msg=n)
