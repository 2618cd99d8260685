"""Debug mode of the exchange (utils/debug.py): finiteness and cross-rank bit identity."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402


def _net():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.ReLU(), torch.nn.Linear(32, 4))


def _body(rank, world, diverge):
    from grace_amd import grace_from_params
    from grace_amd.parallel.optimizer import DistributedOptimizer
    from grace_amd.utils.debug import DivergenceError, ExchangeChecker

    net = _net()
    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.3, "memory": "residual",
                             "communicator": "allgather", "world_size": world})
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), grc,
                               named_parameters=net.named_parameters())
    opt.engine.debug = ExchangeChecker(grc.comm)
    if diverge and rank == 1:
        orig = grc.compressor.decompress_aggregate

        def bad(per_rank, ctx, w):
            return orig(per_rank, ctx, w) * 1.0001  # a rank-local corruption

        grc.compressor.decompress_aggregate = bad
    x = torch.randn(8, 16, generator=torch.Generator().manual_seed(rank))
    opt.zero_grad()
    net(x).sum().backward()
    if diverge:
        with pytest.raises(DivergenceError):
            opt.synchronize()
    else:
        opt.synchronize()
        assert opt.engine.debug.checked == len(opt.engine.buckets)


def test_debug_clean_run_gloo():
    run_distributed(_body, 2, False)


def test_debug_detects_divergence_gloo():
    run_distributed(_body, 2, True)


def test_debug_detects_nonfinite():
    from grace_amd.utils.debug import ExchangeChecker

    with pytest.raises(FloatingPointError):
        ExchangeChecker().check_bucket("b", torch.tensor([1.0, float("nan")]))
