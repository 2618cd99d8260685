"""GPU integration: engine + HIP graphs + native RCCL runtime + DDP hook on one MI355X."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _net():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(3, 16, 3, padding=1), nn.BatchNorm2d(16), nn.ReLU(), nn.AdaptiveAvgPool2d(1),
                         nn.Flatten(), nn.Linear(16, 10)).cuda()


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(8, 3, 16, 16, generator=g).cuda(), torch.randint(0, 10, (8,), generator=g).cuda()


def test_engine_topk_matches_manual_step_loop():
    """Bucketed, stream-overlapped engine == reference-style per-tensor grc.step loop."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.comm import LocalComm

    p = {"compressor": "topk", "compress_ratio": 0.1, "memory": "residual", "communicator": "allgather"}
    m1, m2 = _net(), _net()
    x, y = _data()
    grc1 = grace_from_params(p, comm=LocalComm())
    o1 = torch.optim.SGD(m1.parameters(), lr=0.1)
    o2 = DistributedOptimizer(torch.optim.SGD(m2.parameters(), lr=0.1), grace_from_params(p, comm=LocalComm()),
                              named_parameters=m2.named_parameters(), bucket_cap_mb=0.001)
    for _ in range(3):
        o1.zero_grad()
        F.cross_entropy(m1(x), y).backward()
        for n, prm in m1.named_parameters():
            prm.grad.copy_(grc1.step(prm.grad, n))
        o1.step()
        o2.zero_grad()
        F.cross_entropy(m2(x), y).backward()
        o2.step()
    torch.cuda.synchronize()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_graphed_step_equals_eager():
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.comm import LocalComm
    from grace_amd.parallel.graph import GraphedStep

    p = {"compressor": "topk", "compress_ratio": 0.1, "memory": "residual", "communicator": "allgather"}
    x, y = _data()
    models, outs = [], []
    for graphed in (False, True):
        m = _net()
        o = DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.5),
                                 grace_from_params(p, comm=LocalComm()), named_parameters=m.named_parameters())

        def step():
            o.zero_grad()
            loss = F.cross_entropy(m(x), y)
            loss.backward()
            o.step()
            return loss

        # GraphedStep runs 3 eager warm-up steps and captures (does not execute) the 4th
        run = GraphedStep(step, warmup=3) if graphed else None
        if not graphed:
            for _ in range(3):
                step()
        for _ in range(5):
            (run or step)()
        torch.cuda.synchronize()
        models.append(m)
    for a, b in zip(models[0].parameters(), models[1].parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("overlap", [False, True])
def test_gather_mode_equals_accumulate_mode(overlap):
    """zero_grad(set_to_none=True): fresh gradients are handed over and copied into the buckets
    by the native gather kernel (one launch per bucket) -- identical training to the
    memset + in-place-accumulate mode, also with the compress side stream and a graph."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.comm import LocalComm
    from grace_amd.parallel.graph import GraphedStep

    p = {"compressor": "topk", "compress_ratio": 0.2, "memory": "residual", "communicator": "allgather"}
    x, y = _data()
    res = []
    for none in (False, True):
        m = _net().to(memory_format=torch.channels_last)
        opt = DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9),
                                   grace_from_params(p, comm=LocalComm()), named_parameters=m.named_parameters(),
                                   bucket_cap_mb=0.002, overlap=overlap)

        def step():
            opt.zero_grad(set_to_none=none)
            loss = F.cross_entropy(m(x.contiguous(memory_format=torch.channels_last)), y)
            loss.backward()
            opt.step()
            return loss

        for _ in range(2):
            step()
        g = GraphedStep(step, warmup=2)
        for _ in range(3):
            g()
        torch.cuda.synchronize()
        res.append(torch.cat([q.detach().reshape(-1) for q in m.parameters()]))
    # MIOpen's backward-weight kernels may reduce with atomics: equal up to fp32 rounding
    torch.testing.assert_close(res[1], res[0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("channels_last", [False, True])
def test_bf16_working_weights_match_autocast_gpu(channels_last):
    """Native path: batched bf16 refresh kernel + bf16-widening gather == plain autocast
    (channels_last: dense, non-contiguous conv masters as in bench.py)."""
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_engine import _mp_train

    a = _mp_train("cuda", False, channels_last=channels_last)
    b = _mp_train("cuda", True, channels_last=channels_last)
    torch.testing.assert_close(b.cpu(), a.cpu(), rtol=1e-4, atol=1e-5)
