"""Communicator semantics for W = 4 simulated in ONE process (parallel/loopback.py): fast
coverage of the survey 2.13 compatibility matrix plus the optimizer/engine path, next to
the real multi-process gloo tests (test_distributed_gloo.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(__file__))
import oracles as O  # noqa: E402
from grace_amd import grace_from_params  # noqa: E402
from grace_amd.parallel.loopback import run_ranks  # noqa: E402

W = 4


def _data(rank, seed=0, shape=(23, 19)):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(100 * seed + rank))


def _run(params, name="w", seed=0):
    def fn(rank, comm):
        grc = grace_from_params(dict(params, world_size=W), comm=comm)
        return grc.step(_data(rank, seed), name)

    outs = run_ranks(fn, W)
    for o in outs[1:]:
        assert torch.equal(o, outs[0]), "ranks disagree"
    return outs[0]


def test_loopback_matrix_w4():
    xs = [_data(r) for r in range(W)]
    mean = sum(xs) / W
    for comm in ("allreduce", "allgather", "broadcast"):
        torch.testing.assert_close(_run({"compressor": "none", "communicator": comm}), mean)
    exp = sum(O.topk(t, 0.1) for t in xs) / W
    torch.testing.assert_close(_run({"compressor": "topk", "compress_ratio": 0.1, "communicator": "allgather"}), exp)
    exp = sum(O.threshold(t, 0.8) for t in xs) / W
    torch.testing.assert_close(_run({"compressor": "threshold", "threshold": 0.8, "communicator": "allgather"}), exp)
    a = _run({"compressor": "randomk", "compress_ratio": 0.2, "communicator": "allreduce"}, "rk")
    b = _run({"compressor": "randomk", "compress_ratio": 0.2, "communicator": "allgather"}, "rk")
    torch.testing.assert_close(a, b)
    exp = O.signsgd_vote(xs)
    torch.testing.assert_close(_run({"compressor": "signsgd", "communicator": "allreduce"}), exp)
    out = _run({"compressor": "qsgd", "quantum_num": 15, "communicator": "allreduce"}, "q")
    assert (out - mean).abs().max() <= max(t.norm() for t in xs) / 15 * (1 + 1e-4)
    out = _run({"compressor": "powersgd", "compress_rank": 2, "memory": "powersgd", "communicator": "allreduce"},
               "ps")
    assert torch.isfinite(out).all()
    out = _run({"compressor": "dgc", "memory": "dgc", "gradient_clipping": True, "communicator": "allgather",
                "compress_ratio": 0.05}, "dg")
    assert torch.isfinite(out).all()


def test_loopback_optimizer_keeps_replicas_identical():
    from grace_amd.parallel.optimizer import DistributedOptimizer

    def fn(rank, comm):
        net = torch.nn.Sequential(torch.nn.Linear(12, 24), torch.nn.Tanh(), torch.nn.Linear(24, 3))
        with torch.no_grad():  # consistent init (the global RNG is shared by the rank threads)
            for p in net.parameters():
                comm.broadcast(p.data, 0)
        grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.2, "memory": "residual",
                                 "communicator": "allgather", "world_size": W}, comm=comm)
        opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.05, momentum=0.9), grc,
                                   named_parameters=net.named_parameters(), bucket_cap_mb=0.001)
        for s in range(3):
            x = torch.randn(16, 12, generator=torch.Generator().manual_seed(10 * s + rank))
            opt.zero_grad()
            net(x).pow(2).sum().backward()
            opt.step()
        return torch.cat([p.detach().reshape(-1) for p in net.parameters()]), len(opt.engine.buckets)

    outs = run_ranks(fn, W)
    assert outs[0][1] > 1  # several buckets exercised
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0])
