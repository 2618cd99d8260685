"""FusedSGD: torch.optim.SGD semantics (CPU: functional path; GPU: native kernel)."""
import pytest
import torch

from grace_amd.parallel import FusedSGD

CASES = [dict(momentum=0.0), dict(momentum=0.9), dict(momentum=0.9, nesterov=True, weight_decay=1e-2),
         dict(momentum=0.5, dampening=0.3, weight_decay=5e-4), dict(momentum=0.9, maximize=True)]


def _params(dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 3, 7, 7), (1000, 2048), (7,), (1,), (5, 33), (4097,)]
    ps = [torch.randn(s, generator=g).to(dev) for s in shapes]
    ps[0] = ps[0].contiguous(memory_format=torch.channels_last)  # dense, non-contiguous master
    return ps


def _run(opt_cls, dev, kw, steps=4):
    ps = [p.clone().requires_grad_(True) for p in _params(dev)]
    opt = opt_cls(ps, lr=0.1, **kw)
    g = torch.Generator().manual_seed(1)
    for _ in range(steps):
        for p in ps:
            p.grad = torch.randn(p.shape, generator=g).to(dev).contiguous(memory_format=torch.preserve_format)
            if p.dim() == 4:
                p.grad = p.grad.contiguous(memory_format=torch.channels_last)
        opt.step()
    return ps, opt


@pytest.mark.parametrize("kw", CASES)
def test_fused_sgd_matches_torch_cpu(kw):
    a, _ = _run(torch.optim.SGD, "cpu", kw)
    b, opt = _run(FusedSGD, "cpu", kw)
    for x, y in zip(a, b):
        torch.testing.assert_close(y, x)


def test_fused_sgd_state_dict_is_sgd_compatible():
    _, opt = _run(FusedSGD, "cpu", dict(momentum=0.9))
    sd = opt.state_dict()
    ref = torch.optim.SGD(_params("cpu"), lr=0.1, momentum=0.9)
    ref.load_state_dict(sd)
    assert all("momentum_buffer" in v for v in sd["state"].values())


@pytest.mark.gpu
@pytest.mark.parametrize("kw", CASES)
def test_fused_sgd_native_matches_torch_gpu(kw):
    a, _ = _run(torch.optim.SGD, "cuda", kw)
    b, _ = _run(FusedSGD, "cuda", kw)
    for x, y in zip(a, b):
        assert y.stride() == x.stride()
        torch.testing.assert_close(y, x, rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_fused_sgd_writes_bf16_working_copies_gpu():
    import torch.nn as nn
    from grace_amd.parallel.precision import BF16Weights

    torch.manual_seed(0)
    net = nn.Sequential(nn.Conv2d(3, 16, 3), nn.Flatten(), nn.LazyLinear(4)).cuda()
    net(torch.randn(2, 3, 8, 8, device="cuda"))
    net = net.to(memory_format=torch.channels_last)
    w = BF16Weights(net)
    masters = list(w.master_parameters(net))
    opt = FusedSGD(masters, lr=0.5, momentum=0.9)
    opt.attach_working_copies(w)
    for p in masters:
        p.grad = torch.randn_like(p)
    opt.step()
    for _, _, master, work in w.entries:
        torch.testing.assert_close(work, master.to(torch.bfloat16), rtol=0, atol=0)
