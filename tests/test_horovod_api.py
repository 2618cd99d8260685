"""Horovod-style surface on CPU ranks (gloo, W = 2): mpi_ops handles, variable-size allgather,
sparse (embedding) gradients through DistributedOptimizer, optimizer-state materialisation.

Reference surface: patch_files/horovod/torch/mpi_ops.py:57-439 and
patch_files/horovod/torch/__init__.py:46-403 (IndexedSlices handling for TF at
patch_files/horovod/tensorflow/__init__.py:62-73 is the model for the sparse path).
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402


def _mpi_ops_body(rank, world):
    import grace_amd.torch as hvd

    assert hvd.size() == world and hvd.rank() == rank
    t = torch.full((3, 2), float(rank + 1))
    h = hvd.allreduce_async(t, average=True)
    out = hvd.synchronize(h)
    torch.testing.assert_close(out, torch.full((3, 2), (world + 1) / 2))
    assert torch.equal(t, torch.full((3, 2), float(rank + 1)))  # out-of-place variant
    s = torch.full((4,), float(rank + 1))
    hvd.allreduce_(s, average=False)
    torch.testing.assert_close(s, torch.full((4,), float(sum(range(1, world + 1)))))
    # variable first dimension
    g = hvd.allgather(torch.full((rank + 1, 3), float(rank)))
    exp = torch.cat([torch.full((r + 1, 3), float(r)) for r in range(world)])
    assert torch.equal(g, exp)
    h = hvd.allgather_async(torch.arange(2 * rank + 1))
    assert isinstance(hvd.poll(h), bool)
    got = hvd.synchronize(h)
    assert torch.equal(got, torch.cat([torch.arange(2 * r + 1) for r in range(world)]))
    b = torch.full((5,), float(rank))
    hvd.broadcast_(b, root_rank=1)
    assert torch.equal(b, torch.full((5,), 1.0))


def test_mpi_ops_gloo():
    run_distributed(_mpi_ops_body, 2)


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.emb = torch.nn.Embedding(50, 8, sparse=True)
        self.fc = torch.nn.Linear(8, 4)

    def forward(self, idx):
        return self.fc(self.emb(idx).mean(1))


def _sparse_body(rank, world):
    from grace_amd import grace_from_params
    from grace_amd.parallel.optimizer import DistributedOptimizer, broadcast_optimizer_state, broadcast_parameters

    torch.manual_seed(0)
    net = _Net()
    broadcast_parameters(net.state_dict())
    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.5, "memory": "residual",
                             "communicator": "allgather", "world_size": world})
    opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1, momentum=0.9), grc,
                               named_parameters=net.named_parameters(), sparse_params=["emb.weight"])
    broadcast_optimizer_state(opt)  # materialises momentum buffers on every rank first
    assert len(opt._opt.state_dict()["state"]) > 0
    idx = torch.tensor([[rank, 10 + rank, 20], [3, 4, 5 + rank]])
    opt.zero_grad()
    net(idx).sum().backward()
    local = net.emb.weight.grad.coalesce()
    opt.synchronize()
    g = net.emb.weight.grad
    assert g.is_sparse
    # every rank holds the same averaged sparse gradient
    dense = g.to_dense()
    outs = [torch.empty_like(dense) for _ in range(world)]
    dist.all_gather(outs, dense)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    allg = [torch.empty_like(dense) for _ in range(world)]
    dist.all_gather(allg, local.to_dense())
    torch.testing.assert_close(dense, sum(allg) / world)
    with opt.skip_synchronize():
        opt.step()
    # parameters stay identical across ranks after the step
    w = net.emb.weight.detach().clone()
    ws = [torch.empty_like(w) for _ in range(world)]
    dist.all_gather(ws, w)
    assert torch.equal(ws[0], ws[1])


def test_sparse_embedding_gradients_gloo():
    run_distributed(_sparse_body, 2)
