"""CPU checks of the weight-gradient plumbing (grace_amd/ops/wgrad.py): the split-gradient conv
falls back to nn.Conv2d semantics off the GPU, the engine marks bucket views, and gradients
written into a bucket view reach AccumulateGrad as a stealable alias."""
import torch
import torch.nn as nn

from grace_amd.ops import wgrad


def test_split_conv_cpu_is_conv2d():
    torch.manual_seed(0)
    a = wgrad.Conv2dSplitGrad(4, 6, 3, stride=2, padding=1, bias=False)
    b = nn.Conv2d(4, 6, 3, stride=2, padding=1, bias=False)
    b.load_state_dict(a.state_dict())
    assert set(a.state_dict()) == {"weight"}
    x = torch.randn(2, 4, 9, 9)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = a(xa), b(xb)
    torch.testing.assert_close(ya, yb)
    ya.sum().backward()
    yb.sum().backward()
    torch.testing.assert_close(xa.grad, xb.grad)
    torch.testing.assert_close(a.weight.grad, b.weight.grad)


def test_fork_is_inline_on_cpu():
    t = torch.randn(3)
    with wgrad.fork(t) as side:
        assert side is False


def test_into_target_writes_and_returns_fresh_alias():
    bucket = torch.zeros(20)
    view = bucket[4:16].view(3, 4)
    dw = torch.arange(12, dtype=torch.float32).view(3, 4)
    out = wgrad.into_target(dw, view)
    assert out.data_ptr() == view.data_ptr() and out is not view
    torch.testing.assert_close(bucket[4:16], dw.flatten())
    assert wgrad.into_target(dw, None) is dw


def test_engine_marks_bucket_views_and_steal_keeps_them():
    from grace_amd import grace_from_params
    from grace_amd.parallel.engine import GraceEngine

    model = nn.Sequential(nn.Linear(5, 7), nn.Linear(7, 3))
    grc = grace_from_params({"compressor": "none", "memory": "none", "communicator": "allreduce",
                             "world_size": 1})
    eng = GraceEngine(list(model.named_parameters()), grc, overlap=False)
    views = {id(p): p._grace_grad_view for p in model.parameters()}
    for p in model.parameters():
        p.grad = None
        assert wgrad.grad_target(p) is views[id(p)]
    # a producer that writes the gradient into the view and returns an alias: AccumulateGrad
    # steals the alias, so .grad shares the bucket memory
    w = model[0].weight

    class Producer(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            return x @ w.t()

        @staticmethod
        def backward(ctx, g):
            return None, wgrad.into_target(torch.full_like(w, 2.0), wgrad.grad_target(w))

    Producer.apply(torch.randn(2, 5), w).sum().backward()
    assert w.grad.data_ptr() == views[id(w)].data_ptr()
    assert torch.all(views[id(w)] == 2.0)
    eng.remove()
    assert not hasattr(w, "_grace_grad_view")


def test_only_engine_parameters_may_fork():
    """weight gradients go to the side stream only for parameters whose consumer joins it: the
    engine tags its own (and untags on remove), DDP-managed ones are never tagged"""
    from grace_amd import grace_from_params
    from grace_amd.parallel.ddp_hook import mark_ddp_params
    from grace_amd.parallel.engine import GraceEngine

    model = nn.Sequential(nn.Linear(5, 7), nn.Linear(7, 3))
    assert not any(wgrad.joinable(p) for p in model.parameters())  # plain model: in line
    grc = grace_from_params({"compressor": "none", "memory": "none", "communicator": "allreduce",
                             "world_size": 1})
    eng = GraceEngine(list(model.named_parameters()), grc, overlap=False)
    assert all(wgrad.joinable(p) for p in model.parameters())
    eng.remove()
    assert not any(wgrad.joinable(p) for p in model.parameters())
    wgrad.mark_joinable(model.parameters())
    mark_ddp_params(model.parameters())
    assert not any(wgrad.joinable(p) for p in model.parameters())
