"""PowerSGD under the engine: ONE P and ONE Q all-reduce per step for the whole model.

SURVEY.md 2.11 (row dist/compressor/powersgd.py:46,51) prescribes two matrix collectives per step
for the whole model instead of the reference's two per matrix
(/root/reference/grace_dl/dist/compressor/powersgd.py:45-52).  Here a VGG-16-shaped model (3x3
convs + a large fc stack, scaled down to run on CPU) is split over several buckets; the engine's
step-level exchange must issue exactly 2 matrix all-reduces per step, and its result must equal
the per-bucket immediate exchange (same math, different batching).
"""
import os
import sys

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402


def _vgg_like(seed=0):
    torch.manual_seed(seed)
    c = [8, 8, "M", 16, 16, "M", 32, 32, 32, "M"]
    layers, cin = [], 3
    for v in c:
        if v == "M":
            layers.append(nn.MaxPool2d(2))
        else:
            layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU()]
            cin = v
    return nn.Sequential(*layers, nn.Flatten(), nn.Linear(32 * 2 * 2, 256), nn.ReLU(), nn.Linear(256, 256),
                         nn.ReLU(), nn.Linear(256, 10))


class CountingComm:
    """Wraps a Comm and records the numel of every all-reduce it issues."""

    def __init__(self, inner):
        self.inner = inner
        self.rank, self.world_size = inner.rank, inner.world_size
        self.reduces = []

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def all_reduce(self, t, op="sum", async_op=False):
        self.reduces.append(int(t.numel()))
        return self.inner.all_reduce(t, op, async_op)


def _train(rank, world, step_level, steps=3):
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.comm import LocalComm, TorchComm

    comm = CountingComm(TorchComm() if world > 1 else LocalComm())
    grc = grace_from_params({"compressor": "powersgd", "compress_rank": 2, "memory": "powersgd",
                             "communicator": "allreduce", "world_size": world}, comm=comm)
    model = _vgg_like()
    opt = DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.5), grc,
                               named_parameters=model.named_parameters(), bucket_cap_mb=0.1,
                               overlap=False, group_collectives=False)
    comp = grc.compressor
    comp.enable_step_level(step_level)
    assert len(opt.engine.buckets) >= 3, len(opt.engine.buckets)
    per_step = []
    for s in range(steps):
        g = torch.Generator().manual_seed(100 * s + rank)
        x, y = torch.randn(4, 3, 16, 16, generator=g), torch.randint(0, 10, (4,), generator=g)
        before, nred = comp.matrix_collectives, len(comm.reduces)
        opt.zero_grad()
        F.cross_entropy(model(x), y).backward()
        opt.step()
        per_step.append((comp.matrix_collectives - before, len(comm.reduces) - nred))
    return model, per_step, len(opt.engine.buckets)


def _body(rank, world):
    m_step, counts, nb = _train(rank, world, step_level=True)
    m_buck, counts_b, _ = _train(rank, world, step_level=False)
    # per-bucket immediate exchange: two per bucket that holds a matrix
    mb = counts_b[0][0] // 2
    assert mb >= 2 and all(mat == 2 * mb for mat, _ in counts_b), (counts_b, nb)
    nvec = counts_b[0][1] - 2 * mb  # buckets holding 1-D segments (biases): one all-reduce each
    assert nvec >= 1
    for mat, total in counts:
        assert mat == 2, f"step-level PowerSGD issued {mat} matrix all-reduces in one step"
        assert total == 2 + nvec, (total, nvec)
    for a, b in zip(m_step.parameters(), m_buck.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # the data-parallel invariant: identical replicas
    for p in m_step.parameters():
        t = p.detach().contiguous()
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        assert all(torch.equal(o, out[0]) for o in out)


def test_powersgd_two_matrix_allreduces_per_step_gloo():
    run_distributed(_body, 2)


def test_powersgd_step_level_single_process_matches_per_bucket():
    """W = 1 (no collectives): the deferred step-level exchange trains exactly like the
    per-bucket immediate one, including the PowerSGD residual carried across steps."""
    m1, c1, _ = _train(0, 1, True)
    m2, c2, _ = _train(0, 1, False)
    assert all(mat == 0 for mat, _ in c1 + c2)
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-7)


def test_powersgd_pqt_scale_folds_average():
    from grace_amd.ops import powersgd as PS
    from grace_amd.ops.layout import SegmentLayout

    torch.manual_seed(0)
    lay = SegmentLayout.from_tensors([torch.empty(6, 5), torch.empty(7)])
    plan = PS.plan_for(lay, 2)
    p = torch.randn(plan.p_total)
    q = torch.randn(plan.q_total)
    a = torch.zeros(lay.total)
    b = torch.zeros(lay.total)
    PS.pqt(p, q, plan, a)
    PS.pqt(p, q, plan, b, scale=0.25)
    torch.testing.assert_close(b, a * 0.25)


def test_deferred_residual_ops_match_eager_update_cpu():
    """ops.powersgd: the deferred residual -- mq(comp_r=M_prev, lazy=(P, Q, s)) -- compensates with
    exactly the residual the eager pqt(resid=...) update would have left (same float ops on the
    PyTorch path), and pqt(out=None, resid=...) materialises it."""
    from grace_amd.ops import powersgd as PS
    from grace_amd.ops.layout import SegmentLayout

    g = torch.Generator().manual_seed(0)
    shapes = [(30, 20), (7,), (8, 3, 3, 3)]
    lay = SegmentLayout.from_tensors([torch.empty(s) for s in shapes])
    plan = PS.plan_for(lay, 2)
    m_prev = torch.randn(lay.total, generator=g)
    p = torch.randn(plan.p_total, generator=g)
    q = torch.randn(plan.q_total, generator=g)
    s = 0.25
    # eager: r = M_prev - s P Q^T on the matrix segments (pqt), then M = 0.9 r + 1.0 x
    r_eager = m_prev.clone()
    PS.pqt(p, q, plan, torch.empty(lay.total), resid=r_eager, scale=s)
    x = torch.randn(lay.total, generator=g)
    q_new = torch.randn(plan.q_total, generator=g)
    out_e = r_eager.clone()
    p_e = PS.mq(x, q_new, plan, comp_r=r_eager.clone(), beta=0.9, gamma=1.0, xout=out_e)
    out_d = m_prev.clone()
    p_d = PS.mq(x, q_new, plan, comp_r=m_prev.clone(), beta=0.9, gamma=1.0, xout=out_d, lazy=(p, q, s))
    for (xo, n, mm, rr, po, qo) in plan.mats:
        assert torch.equal(out_e[xo:xo + n * mm], out_d[xo:xo + n * mm])
    assert torch.equal(p_e, p_d)
    r_mat = m_prev.clone()
    PS.pqt(p, q, plan, None, resid=r_mat, scale=s)  # materialise only
    assert torch.equal(r_mat, r_eager)


def test_powersgd_memory_state_dict_materialises_copy_cpu():
    """PowerSGDMemory with a deferred entry: state_dict() returns M - s P Q^T and leaves the live
    buffer (M) untouched; materialize() applies it in place; load_state_dict clears the deferral."""
    from grace_amd.memory.powersgd import PowerSGDMemory
    from grace_amd.ops import powersgd as PS
    from grace_amd.ops.layout import SegmentLayout

    g = torch.Generator().manual_seed(1)
    lay = SegmentLayout.from_tensors([torch.empty(12, 5), torch.empty(3)])
    plan = PS.plan_for(lay, 2)
    mem = PowerSGDMemory(compress_rank=2)
    m = torch.randn(lay.total, generator=g)
    mem.residuals["b"] = m.clone()
    p, q = torch.randn(plan.p_total, generator=g), torch.randn(plan.q_total, generator=g)
    mem.lazy["b"] = (p, q, 0.5, plan)
    want = m.clone()
    PS.pqt(p, q, plan, None, resid=want, scale=0.5)
    sd = mem.state_dict()
    assert torch.equal(sd["residuals"]["b"], want)
    assert torch.equal(mem.residuals["b"], m) and "b" in mem.lazy
    mem.materialize()
    assert torch.equal(mem.residuals["b"], want) and not mem.lazy
    mem.lazy["b"] = (p, q, 0.5, plan)
    mem.load_state_dict(sd)
    assert not mem.lazy and torch.equal(mem.residuals["b"], want)
