"""W = 2 ranks on ONE MI355X (gloo carries the GPU payloads): the native HIP codec kernels and
the bucketed engine in a real multi-rank exchange -- multi-rank decode (W payloads), majority
votes, shared-scale QSGD, PowerSGD's averaged P/Q, variable-size payloads, cross-rank identity.
(RCCL refuses two ranks on one GPU; the 8-GPU RCCL run is the driver's scaling bench.)"""
import os
import sys

import pytest
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402
from test_distributed_gloo import _body, _same_on_all_ranks  # noqa: E402

pytestmark = pytest.mark.gpu


def test_communicators_two_ranks_gpu():
    run_distributed(_body, 2, "cuda")


def _engine_body(rank, world):
    import torch.nn as nn
    import torch.nn.functional as F

    from grace_amd import grace_from_params
    from grace_amd.ops.bnact import BatchNormAct2d
    from grace_amd.parallel import DistributedOptimizer, FusedSGD, broadcast_parameters
    from grace_amd.parallel.precision import BF16Weights

    dev = torch.device("cuda", 0)
    torch.manual_seed(rank)  # different init per rank: broadcast must fix it
    net = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1, bias=False), BatchNormAct2d(16, relu=True),
                        nn.Conv2d(16, 32, 3, stride=2, padding=1, bias=False), BatchNormAct2d(32, relu=True),
                        nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10)).to(dev)
    net = net.to(memory_format=torch.channels_last)
    broadcast_parameters(net.state_dict(), root_rank=0)
    w = BF16Weights(net)
    named = list(w.named_master_parameters(net))
    for comp in ({"compressor": "topk", "compress_ratio": 0.1, "memory": "residual", "communicator": "allgather"},
                 {"compressor": "efsignsgd", "lr": 0.1, "memory": "efsignsgd", "communicator": "allreduce"},
                 {"compressor": "qsgd", "quantum_num": 127, "communicator": "allreduce"}):
        grc = grace_from_params(dict(comp, world_size=world))
        opt = DistributedOptimizer(FusedSGD([p for _, p in named], lr=0.05, momentum=0.9), grc,
                                   named_parameters=named, weights=w, bucket_cap_mb=0.01)
        g = torch.Generator().manual_seed(100 + rank)  # rank-specific data
        for _ in range(3):
            x = torch.randn(8, 3, 16, 16, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
            y = torch.randint(0, 10, (8,), generator=g).to(dev)
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(net(x), y)
            loss.backward()
            opt.step()
        torch.cuda.synchronize()
        for _, p in named:
            _same_on_all_ranks(p)
        opt.engine.remove()


def test_engine_two_ranks_gpu():
    run_distributed(_engine_body, 2)
