"""Training-integration tests on CPU: DistributedOptimizer engine, DDP comm hook, broadcasts."""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402


def _model(seed=0):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(20, 64), nn.ReLU(), nn.Linear(64, 32), nn.ReLU(), nn.Linear(32, 5))


def _batch(rank, seed=0):
    g = torch.Generator().manual_seed(100 * seed + rank)
    return torch.randn(16, 20, generator=g), torch.randint(0, 5, (16,), generator=g)


def test_engine_none_equals_plain_sgd_single_process():
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer

    m1, m2 = _model(), _model()
    o1 = torch.optim.SGD(m1.parameters(), lr=0.1, momentum=0.9)
    grc = grace_from_params({"compressor": "none", "communicator": "allreduce"})
    o2 = DistributedOptimizer(torch.optim.SGD(m2.parameters(), lr=0.1, momentum=0.9), grc,
                              named_parameters=m2.named_parameters(), bucket_cap_mb=0.001)
    assert len(o2.engine.buckets) > 1
    for s in range(4):
        x, y = _batch(0, s)
        o1.zero_grad()
        F.cross_entropy(m1(x), y).backward()
        o1.step()
        o2.zero_grad()
        F.cross_entropy(m2(x), y).backward()
        o2.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b)


def test_backward_passes_per_step_accumulates():
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer

    m1, m2 = _model(), _model()
    o1 = torch.optim.SGD(m1.parameters(), lr=0.1)
    o2 = DistributedOptimizer(torch.optim.SGD(m2.parameters(), lr=0.1), grace_from_params({}),
                              named_parameters=m2.named_parameters(), backward_passes_per_step=2)
    o1.zero_grad()
    o2.zero_grad()
    for s in range(2):
        x, y = _batch(0, s)
        F.cross_entropy(m1(x), y).backward()
        F.cross_entropy(m2(x), y).backward()
    o1.step()
    o2.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b)


def test_zero_grad_race_guard():
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer

    m = _model()
    o = DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), grace_from_params({}),
                             named_parameters=m.named_parameters())
    x, y = _batch(0)
    F.cross_entropy(m(x), y).backward()
    with pytest.raises(AssertionError):
        o.zero_grad()
    o.step()
    o.zero_grad()


def _dp_body(rank, world, params, group=False):
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer, broadcast_parameters

    m = _model(seed=rank)  # different init on purpose: broadcast must fix it
    broadcast_parameters(m.state_dict(), root_rank=0)
    ref = _model(seed=0)
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b)
    grc = grace_from_params(dict(params, world_size=world))
    opt = DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.05), grc, named_parameters=m.named_parameters(),
                               bucket_cap_mb=0.002, group_collectives=group)
    assert opt.engine.grouped == bool(group)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.05)
    for s in range(3):
        x, y = _batch(rank, s)
        opt.zero_grad()
        F.cross_entropy(m(x), y).backward()
        opt.step()
        if params.get("compressor", "none") == "none":
            # reference: average of all ranks' gradients
            ref_opt.zero_grad()
            for r in range(world):
                xr, yr = _batch(r, s)
                (F.cross_entropy(ref(xr), yr) / world).backward()
            ref_opt.step()
    # replicas identical on every rank
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    out = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(out, flat)
    for o in out[1:]:
        assert torch.equal(o, out[0])
    if params.get("compressor", "none") == "none":
        for a, b in zip(m.parameters(), ref.parameters()):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("params", [
    {"compressor": "none", "communicator": "allreduce"},
    {"compressor": "topk", "compress_ratio": 0.1, "memory": "residual", "communicator": "allgather"},
    {"compressor": "efsignsgd", "lr": 0.1, "memory": "efsignsgd", "communicator": "allreduce"},
    {"compressor": "qsgd", "quantum_num": 15, "communicator": "allreduce"},
    {"compressor": "powersgd", "compress_rank": 2, "memory": "powersgd", "communicator": "allreduce"},
])
def test_distributed_optimizer_gloo(params):
    run_distributed(_dp_body, 2, params)


@pytest.mark.parametrize("params", [
    {"compressor": "none", "communicator": "allreduce"},
    {"compressor": "topk", "compress_ratio": 0.1, "memory": "residual", "communicator": "allgather"},
    {"compressor": "powersgd", "compress_rank": 2, "memory": "powersgd", "communicator": "allreduce"},
    {"compressor": "dgc", "compress_ratio": 0.1, "memory": "dgc", "communicator": "allgather"},
])
def test_grouped_collectives_gloo(params):
    """GroupedComm: every bucket's collective deferred to synchronize() and issued together
    (one RCCL group on the native runtime); blocking in-compress collectives (PowerSGD) flush
    first.  Same results as the ungrouped path (plain SGD reference for None)."""
    run_distributed(_dp_body, 2, params, True)


def _ddp_body(rank, world):
    from grace_amd import grace_from_params
    from grace_amd.parallel import GraceHookState, grace_comm_hook

    m = _model(seed=0)
    ddp = nn.parallel.DistributedDataParallel(m, bucket_cap_mb=0.002)
    ddp.register_comm_hook(GraceHookState(grace_from_params({"compressor": "none", "world_size": world})),
                           grace_comm_hook)
    ref = _model(seed=0)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.05)
    ref_opt = torch.optim.SGD(ref.parameters(), lr=0.05)
    for s in range(2):
        x, y = _batch(rank, s)
        opt.zero_grad()
        F.cross_entropy(ddp(x), y).backward()
        opt.step()
        ref_opt.zero_grad()
        for r in range(world):
            xr, yr = _batch(r, s)
            (F.cross_entropy(ref(xr), yr) / world).backward()
        ref_opt.step()
    for a, b in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_ddp_comm_hook_gloo():
    run_distributed(_ddp_body, 2)


def _mp_net():
    torch.manual_seed(3)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3, padding=1), torch.nn.BatchNorm2d(8), torch.nn.ReLU(),
                               torch.nn.AdaptiveAvgPool2d(1), torch.nn.Flatten(), torch.nn.Linear(8, 5))


def _mp_train(dev, use_weights, steps=3, channels_last=False):
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.comm import LocalComm
    from grace_amd.parallel.precision import BF16Weights

    net = _mp_net().to(dev)
    if channels_last:  # conv masters become dense-but-not-contiguous (the bench's layout)
        net = net.to(memory_format=torch.channels_last)
    w = BF16Weights(net) if use_weights else None
    named = list(w.named_master_parameters(net)) if w else list(net.named_parameters())
    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.3, "memory": "residual",
                             "communicator": "allgather"}, comm=LocalComm())
    opt = DistributedOptimizer(torch.optim.SGD([p for _, p in named], lr=0.05, momentum=0.9), grc,
                               named_parameters=named, bucket_cap_mb=0.001, weights=w)
    g = torch.Generator().manual_seed(5)
    x, y = torch.randn(6, 3, 8, 8, generator=g).to(dev), torch.randint(0, 5, (6,), generator=g).to(dev)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    for _ in range(steps):
        opt.zero_grad()
        with torch.autocast(torch.device(dev).type, dtype=torch.bfloat16):
            loss = torch.nn.functional.cross_entropy(net(x), y)
        loss.backward()
        opt.step()
    return torch.cat([p.detach().float().reshape(-1) for _, p in named])


def test_bf16_working_weights_match_autocast_cpu():
    """fp32 masters + bf16 working copies == plain autocast (same roundings, fewer kernels)."""
    a = _mp_train("cpu", False)
    b = _mp_train("cpu", True)
    torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)


def test_bf16_working_weights_channels_last_cpu():
    a = _mp_train("cpu", False, channels_last=True)
    b = _mp_train("cpu", True, channels_last=True)
    torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)


def _ddp_net(seed=0):
    torch.manual_seed(seed)
    # every matrix has min(rows, cols) <= 4: PowerSGD rank 4 is then exact (full-rank P Q^T)
    return nn.Sequential(nn.Conv2d(3, 4, 3, padding=1), nn.ReLU(), nn.AdaptiveAvgPool2d(2), nn.Flatten(),
                         nn.Linear(16, 4), nn.ReLU(), nn.Linear(4, 3))


def _ddp_value_body(rank, world, params, kind, defer=False):
    """DDP comm hook == the reference's per-parameter loop ``grc.step(p.grad, name)``
    (examples/dist/CIFAR10-dawndist/core.py:203-206) on the same gradients, 3 steps with memory.
    ``defer``: the hook queues each bucket and ``flush()`` runs the exchanges after backward."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import GraceHookState, grace_comm_hook

    m = _ddp_net()
    ddp = nn.parallel.DistributedDataParallel(m, bucket_cap_mb=0.0002, gradient_as_bucket_view=defer)
    st = GraceHookState(grace_from_params(dict(params, world_size=world)), model=ddp, defer=defer)
    ddp.register_comm_hook(st, grace_comm_hook)
    ref = _ddp_net()
    grc_ref = grace_from_params(dict(params, world_size=world))
    named = list(ref.named_parameters())
    for s in range(3):
        g = torch.Generator().manual_seed(100 * s + rank)
        x, y = torch.randn(8, 3, 6, 6, generator=g), torch.randint(0, 3, (8,), generator=g)
        for p in ddp.parameters():
            p.grad = None
        F.cross_entropy(ddp(x), y).backward()
        if defer:
            assert len(st.pending) >= (1 if s == 0 else 2), (s, len(st.pending))  # queued, not yet exchanged
            st.flush()
            assert not st.pending
        ref.zero_grad()
        F.cross_entropy(ref(x), y).backward()
        exp = [grc_ref.step(p.grad.clone(), n) for n, p in named]  # per-parameter loop (reverse not needed)
        got = [p.grad for p in ddp.module.parameters()]
        for (n, _), a, b in zip(named, got, exp):
            if kind == "exact":
                torch.testing.assert_close(a, b.view_as(a), rtol=1e-5, atol=1e-6, msg=f"{n} step {s}")
            elif kind == "lowrank":  # full-rank PowerSGD: exact up to the CholQR2 rounding
                torch.testing.assert_close(a, b.view_as(a), rtol=1e-3, atol=1e-4 * float(b.abs().max()) + 1e-7,
                                           msg=f"{n} step {s}")
            else:  # stochastic codec: independent seeds per name; the QSGD error bound holds
                assert (a - b.view_as(a)).abs().max() <= 2 * float(b.abs().max()) + 1e-6, n
        # keep both models on the same weights (compare gradients step by step)
        with torch.no_grad():
            for p, q in zip(ddp.module.parameters(), ref.parameters()):
                p.sub_(0.05 * p.grad)
                q.copy_(p)
    # the DP invariant
    for p in ddp.module.parameters():
        t = p.detach().contiguous()
        allv = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        assert all(torch.equal(a, allv[0]) for a in allv)
    assert len(st.layouts) > 1


@pytest.mark.parametrize("params,kind", [
    ({"compressor": "topk", "compress_ratio": 0.3, "memory": "residual", "communicator": "allgather"}, "exact"),
    ({"compressor": "efsignsgd", "lr": 0.1, "memory": "efsignsgd", "communicator": "allreduce"}, "exact"),
    ({"compressor": "qsgd", "quantum_num": 127, "communicator": "allreduce"}, "bounded"),
    ({"compressor": "powersgd", "compress_rank": 4, "memory": "powersgd", "communicator": "allreduce"}, "lowrank"),
])
@pytest.mark.parametrize("world", [2, 3])
def test_ddp_hook_matches_per_parameter_loop_gloo(params, kind, world):
    run_distributed(_ddp_value_body, world, params, kind)


@pytest.mark.parametrize("params,kind", [
    ({"compressor": "topk", "compress_ratio": 0.3, "memory": "residual", "communicator": "allgather"}, "exact"),
    ({"compressor": "powersgd", "compress_rank": 4, "memory": "powersgd", "communicator": "allreduce"}, "lowrank"),
])
def test_deferred_ddp_hook_matches_per_parameter_loop_gloo(params, kind):
    """GraceHookState(defer=True): same gradients as the immediate hook / the per-parameter loop,
    with every bucket's exchange run by flush() after backward (gradient_as_bucket_view)."""
    run_distributed(_ddp_value_body, 2, params, kind, True)


def test_ddp_hook_padded_bucket_keeps_per_parameter_layout():
    """A bucket whose gradient views leave gaps (DDP alignment padding) is packed into the
    per-parameter layout instead of collapsing to one whole-bucket segment."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import GraceHookState, grace_comm_hook
    from grace_amd.parallel.comm import LocalComm

    buf = torch.zeros(40)
    g1, g2 = buf[0:10].view(2, 5), buf[16:36].view(4, 5)  # gap at 10..16, tail 36..40
    p1, p2 = torch.nn.Parameter(torch.zeros(2, 5)), torch.nn.Parameter(torch.zeros(4, 5))
    torch.manual_seed(0)
    g1.copy_(torch.randn(2, 5))
    g2.copy_(torch.randn(4, 5))

    class FakeBucket:
        def index(self):
            return 0

        def buffer(self):
            return buf

        def gradients(self):
            return [g1, g2]

        def parameters(self):
            return [p1, p2]

    params = {"compressor": "topk", "compress_ratio": 0.2, "communicator": "allgather"}
    st = GraceHookState(grace_from_params(params, comm=LocalComm()))
    out = grace_comm_hook(st, FakeBucket()).wait()
    assert st.packed_buckets == 1 and st.layouts[0][0].numels == (10, 20)
    ref = grace_from_params(params, comm=LocalComm())
    torch.testing.assert_close(out[0:10].view(2, 5), ref.step(g1.clone(), "a"))
    torch.testing.assert_close(out[16:36].view(4, 5), ref.step(g2.clone(), "b"))
    assert float(out[10:16].abs().sum()) == 0 and float(out[36:].abs().sum()) == 0


def _ddp_randomk_body(rank, world):
    """Random-K through the DDP hook: every rank must draw the SAME indices (rank-invariant bucket
    names feed the shared seed), so each tensor's averaged gradient has exactly k non-zeros."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import GraceHookState, grace_comm_hook

    m = _ddp_net()
    ddp = nn.parallel.DistributedDataParallel(m, bucket_cap_mb=0.0002)
    ddp.register_comm_hook(GraceHookState(grace_from_params({"compressor": "randomk", "compress_ratio": 0.25,
                                                             "communicator": "allreduce", "world_size": world})),
                           grace_comm_hook)
    for s in range(3):
        g = torch.Generator().manual_seed(100 * s + rank)
        x, y = torch.randn(8, 3, 6, 6, generator=g), torch.randint(0, 3, (8,), generator=g)
        for p in ddp.parameters():
            p.grad = None
        F.cross_entropy(ddp(x), y).backward()
        for p in ddp.module.parameters():
            k = max(1, int(p.numel() * 0.25))
            assert int((p.grad != 0).sum()) <= k, (tuple(p.shape), int((p.grad != 0).sum()), k)


def test_ddp_hook_randomk_shared_indices_gloo():
    run_distributed(_ddp_randomk_body, 2)


def _ddp_views_body(rank, world):
    from grace_amd import grace_from_params
    from grace_amd.parallel import GraceHookState, grace_comm_hook

    m = _model(seed=0)
    ddp = nn.parallel.DistributedDataParallel(m, bucket_cap_mb=0.002, gradient_as_bucket_view=True)
    st = GraceHookState(grace_from_params({"compressor": "none", "world_size": world}), model=ddp)
    ddp.register_comm_hook(st, grace_comm_hook)
    assert all(getattr(p, "_grace_ddp", False) for p in m.parameters())  # marked before any backward
    opt = torch.optim.SGD(ddp.parameters(), lr=0.05)
    for s in range(3):  # DDP rebuilds its buckets after the first iteration
        x, y = _batch(rank, s)
        opt.zero_grad(set_to_none=True)
        F.cross_entropy(ddp(x), y).backward()
        opt.step()
    for p in m.parameters():  # the gradient targets are the CURRENT bucket views
        assert p._grace_grad_view.data_ptr() == p.grad.data_ptr()


def test_ddp_hook_marks_current_bucket_views_gloo():
    run_distributed(_ddp_views_body, 2)


def test_tail_bucket_same_result_as_one_bucket():
    """GraceEngine(tail_bucket=True): the first layer's weight gets a bucket of its own, exchanged
    last; per-tensor Top-K gives the same gradients as with one bucket."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer

    def run(tail):
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.Flatten(),
                                torch.nn.Linear(8 * 6 * 6, 4))
        grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.1, "memory": "residual",
                                 "communicator": "allgather"})
        opt = DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), grc,
                                   named_parameters=list(m.named_parameters()), overlap=False, tail_bucket=tail)
        g = torch.Generator().manual_seed(1)
        for _ in range(3):
            x = torch.randn(5, 3, 8, 8, generator=g)
            opt.zero_grad()
            m(x).square().mean().backward()
            opt.step()
        return opt, [p.detach().clone() for p in m.parameters()]

    o1, a = run(False)
    o2, b = run(True)
    assert len(o1.engine.buckets) == 1 and len(o2.engine.buckets) == 2
    assert o2.engine.buckets[-1].params[0].dim() == 4  # conv weight alone, last
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=0, atol=0)
