"""One-shot xGMI peer-memory all-gather (grace_amd/parallel/xgmi.py, csrc/comm/xgmi_allgather.hip).

On the 1-GPU test box the W = 2 ranks share cuda:0: the HIP IPC handles, the ready-generation
protocol, the slot double-buffering and graph replay are exercised for real (the same code then
reads a peer's HBM over its xGMI link on an 8-GPU node).  Every result is compared with the
inner comm's (gloo) all-gather of the same tensors."""
import os
import sys

import pytest
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402

pytestmark = pytest.mark.gpu


def _xgmi_body(rank, world):
    from grace_amd.parallel.comm import TorchComm
    from grace_amd.parallel.xgmi import XgmiComm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    inner = TorchComm()
    comm = XgmiComm(inner, capacity_mb=1.0)  # construction runs the self-check
    # eager calls of different sizes (both slots, several generations, uneven grid tails)
    g = torch.Generator().manual_seed(rank)
    for n in (16, 4096, 65536 + 48, 250000):
        inp = torch.randint(0, 255, (n,), generator=g, dtype=torch.uint8).to(dev)
        out = torch.empty(world * n, dtype=torch.uint8, device=dev)
        ref = torch.empty_like(out)
        comm.all_gather_into(out, inp)
        inner.all_gather_into(ref, inp)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), f"size {n}"
    assert comm.one_shot_calls == 4
    # too large for the capacity -> inner comm
    big = torch.ones(2 ** 20 + 16, dtype=torch.uint8, device=dev)
    bout = torch.empty(world * big.numel(), dtype=torch.uint8, device=dev)
    comm.all_gather_into(bout, big)
    assert comm.one_shot_calls == 4 and torch.equal(bout, torch.ones_like(bout))
    # graph capture: the generation lives on the device, so replays advance it
    src = torch.zeros(8192, dtype=torch.float32, device=dev)
    dst = torch.empty(world * 8192, dtype=torch.float32, device=dev)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        comm.all_gather_into(dst, src)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        comm.all_gather_into(dst, src)
    for it in range(5):
        src.copy_(torch.arange(8192, device=dev, dtype=torch.float32) * (rank + 1) + it)
        graph.replay()
        torch.cuda.synchronize()
        want = torch.cat([torch.arange(8192, device=dev, dtype=torch.float32) * (r + 1) + it for r in range(world)])
        assert torch.equal(dst, want), f"replay {it}"
    # all-reduce as a one-shot gather + rank-ordered local reduction (sum / max)
    for op in ("sum", "max"):
        t = torch.randn(10000, generator=torch.Generator().manual_seed(40 + rank)).to(dev)
        ref = t.clone()
        calls = comm.one_shot_calls
        comm.all_reduce(t, op)
        inner.all_reduce(ref, op)
        torch.cuda.synchronize()
        assert comm.one_shot_calls == calls + 1
        if world == 2 or op == "max":  # two fp32 terms: order-free, so gloo's sum is bit-comparable
            assert torch.equal(t, ref), op
        else:
            torch.testing.assert_close(t, ref, rtol=1e-6, atol=1e-6)
        same = t.clone()
        dist.broadcast(same, 0)
        assert torch.equal(same, t), "ranks disagree"  # identical bytes reduced in identical order
    comm.check()  # no timed-out waits
    dist.barrier()
    torch.cuda.synchronize()
    comm.close()


def test_xgmi_allgather_two_ranks_one_gpu():
    run_distributed(_xgmi_body, 2, timeout=180)


def test_xgmi_allgather_four_ranks_one_gpu():
    """W = 4 (three peers per puller: the grid's rank dimension, the consumed fan-in)"""
    run_distributed(_xgmi_body, 4, timeout=240)


def test_xgmi_allgather_engine_topk():
    """The bucketed Top-K + Allgather engine at W = 2 with the one-shot comm as the default comm:
    parameters stay identical across ranks and the one-shot path carried the payloads."""
    run_distributed(_xgmi_engine_body, 2, timeout=180)


def _xgmi_engine_body(rank, world):
    import torch.nn as nn
    import torch.nn.functional as F

    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer, broadcast_parameters, set_default_comm
    from grace_amd.parallel.comm import TorchComm
    from grace_amd.parallel.xgmi import XgmiComm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = XgmiComm(TorchComm(), capacity_mb=2.0)
    set_default_comm(comm)
    try:
        torch.manual_seed(rank)
        net = nn.Sequential(nn.Linear(64, 256), nn.ReLU(), nn.Linear(256, 10)).to(dev)
        broadcast_parameters(net.state_dict(), root_rank=0)
        grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.05, "memory": "residual",
                                 "communicator": "allgather", "world_size": world})
        opt = DistributedOptimizer(torch.optim.SGD(net.parameters(), lr=0.1), grc,
                                   named_parameters=net.named_parameters(), overlap=False)
        g = torch.Generator().manual_seed(10 + rank)
        for _ in range(4):
            x = torch.randn(16, 64, generator=g).to(dev)
            y = torch.randint(0, 10, (16,), generator=g).to(dev)
            opt.zero_grad()
            F.cross_entropy(net(x), y).backward()
            opt.step()
        torch.cuda.synchronize()
        assert comm.one_shot_calls > 0
        for p in net.parameters():
            ref = p.detach().clone()
            dist.broadcast(ref, 0)
            assert torch.equal(ref, p.detach())
        comm.check()
        dist.barrier()
        torch.cuda.synchronize()
    finally:
        set_default_comm(None)
        comm.close()


def _xgmi_timeout_body(rank, world):
    """A peer that arrives later than the spin limit: the waiting rank zero-fills that peer's
    rows, raises the fault flag (host-mapped: check() raises without a device sync) and its
    FusedSGD skips the update; the late rank still gets correct data."""
    import time

    from grace_amd.parallel import FusedSGD, health
    from grace_amd.parallel.comm import TorchComm
    from grace_amd.parallel.xgmi import XgmiComm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = XgmiComm(TorchComm(), capacity_mb=1.0, spin_limit=1 << 18)
    health.reset()
    p = torch.nn.Parameter(torch.ones(1024, device=dev))
    opt = FusedSGD([p], lr=0.5)
    inp = torch.full((4096,), rank + 1, dtype=torch.int32, device=dev)
    out = torch.full((world * 4096,), -7, dtype=torch.int32, device=dev)
    dist.barrier()
    if rank == 1:
        time.sleep(4.0)  # far beyond rank 0's spin limit
    comm.all_gather_into(out, inp)
    torch.cuda.synchronize()
    if rank == 0:
        assert torch.equal(out[:4096], inp)
        assert torch.equal(out[4096:], torch.zeros(4096, dtype=torch.int32, device=dev)), "late peer not zero-filled"
        assert health.status()[1] >= 1
        with pytest.raises(health.CommFault):
            comm.check()
        p.grad = torch.ones_like(p)
        opt.step()  # must be skipped while the fault flag is raised
        torch.cuda.synchronize()
        assert torch.equal(p.detach(), torch.ones_like(p))
    else:
        want = torch.cat([torch.full((4096,), r + 1, dtype=torch.int32, device=dev) for r in range(world)])
        assert torch.equal(out, want)
    dist.barrier()
    health.reset()
    p.grad = torch.ones_like(p)
    opt.step()  # fault cleared: the update runs again
    torch.cuda.synchronize()
    assert torch.allclose(p.detach(), torch.full_like(p, 0.5))
    dist.barrier()
    comm.close()


def test_xgmi_peer_timeout_is_fatal_not_silent():
    run_distributed(_xgmi_timeout_body, 2, timeout=180)


def _xgmi_count_body(rank, world):
    """Capacity payloads (Threshold): the one-shot pull copies only each peer's VALID entries
    (count from the peer's in-band header); the decoded result equals the inner comm's."""
    from grace_amd import grace_from_params
    from grace_amd.parallel.comm import TorchComm
    from grace_amd.parallel.xgmi import XgmiComm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = XgmiComm(TorchComm(), capacity_mb=2.0)
    params = {"compressor": "threshold", "threshold": 1.5, "memory": "none", "communicator": "allgather",
              "world_size": world}
    g = torch.Generator().manual_seed(3 + rank)
    for step in range(3):
        x = torch.randn(50000, generator=g).to(dev)
        a = grace_from_params(params, comm=comm).step(x.clone(), "t")
        b = grace_from_params(params, comm=TorchComm()).step(x.clone(), "t")
        torch.cuda.synchronize()
        assert torch.equal(a, b), f"step {step}"
    assert comm.one_shot_calls >= 3
    comm.check()
    dist.barrier()
    torch.cuda.synchronize()
    comm.close()


def test_xgmi_count_aware_capacity_payload():
    run_distributed(_xgmi_count_body, 2, timeout=180)


def _xgmi_direct_body(rank, world):
    """Top-K's payload assembled straight in the exported slot (uncached regions): the gather
    runs without the staging copy and matches the staged path."""
    from grace_amd import grace_from_params
    from grace_amd.parallel.comm import TorchComm
    from grace_amd.parallel.xgmi import XgmiComm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = XgmiComm(TorchComm(), capacity_mb=2.0)
    params = {"compressor": "topk", "compress_ratio": 0.02, "memory": "none", "communicator": "allgather",
              "world_size": world}
    g = torch.Generator().manual_seed(11 + rank)
    for step in range(3):
        x = torch.randn(60000, generator=g).to(dev)
        a = grace_from_params(params, comm=comm).step(x.clone(), "bucket")
        b = grace_from_params(params, comm=TorchComm()).step(x.clone(), "bucket")
        torch.cuda.synchronize()
        assert torch.equal(a, b), f"step {step}"
    if comm._x.uncached:
        assert comm.direct_calls >= 3
    # ranks that DISAGREE on the slot (rank 0 assembles in slot D, rank 1 is staged): every
    # puller reads the slot its peer published, not its own choice
    if comm._direct_ok:
        n = 4096
        pat = torch.arange(n, device=dev, dtype=torch.int32) * (rank + 3) + 17
        inp = comm._x.slot_tensor(n * 4).view(torch.int32) if rank == 0 else pat.clone()
        inp.copy_(pat)
        out = torch.empty(world * n, dtype=torch.int32, device=dev)
        comm._x.all_gather(out.view(torch.uint8), inp.view(torch.uint8), torch.empty(0, 8, dtype=torch.int64))
        torch.cuda.synchronize()
        want = torch.cat([torch.arange(n, device=dev, dtype=torch.int32) * (r + 3) + 17 for r in range(world)])
        assert torch.equal(out, want)
        # a retired owner hands the slot on after _OWNER_IDLE calls by other keys
        comm._slot_owner = None
        assert comm.payload_buffer(64, "old") is not None
        got = [comm.payload_buffer(64, "new") is not None for _ in range(comm._OWNER_IDLE + 2)]
        assert not got[0] and got[-1]
        assert comm.payload_buffer(64, "old") is None
    comm.check()
    dist.barrier()
    torch.cuda.synchronize()
    comm.close()


def test_xgmi_direct_payload_no_staging():
    run_distributed(_xgmi_direct_body, 2, timeout=180)


def _xgmi_whole_step_graph_body(rank, world):
    """The W > 1 measured configuration, rehearsed on one GPU: forward + backward + Top-K 1 %
    exchange (xGMI one-shot all-gather, GroupedComm) + FusedSGD captured as ONE HIP graph and
    replayed 10 times.  Ranks train on different data; after every replay the weights must be
    bit-identical across ranks (the exchange averaged the same decoded gradient everywhere),
    and the device health words must stay clean."""
    import torch.nn.functional as F

    from grace_amd import grace_from_params
    from grace_amd.models import resnet18_cifar
    from grace_amd.parallel import DistributedOptimizer, FusedSGD, broadcast_parameters, set_default_comm
    from grace_amd.parallel.comm import TorchComm
    from grace_amd.parallel.graph import GraphedStep
    from grace_amd.parallel.xgmi import XgmiComm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = XgmiComm(TorchComm(), capacity_mb=8.0, select="probe")
    set_default_comm(comm)
    try:
        torch.manual_seed(0)
        model = resnet18_cifar().to(dev).to(memory_format=torch.channels_last)
        broadcast_parameters(model.state_dict(), root_rank=0)
        grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.01, "memory": "residual",
                                 "communicator": "allgather", "world_size": world})
        opt = DistributedOptimizer(FusedSGD(list(model.parameters()), lr=0.02, momentum=0.5), grc,
                                   named_parameters=list(model.named_parameters()), overlap=False)
        g = torch.Generator().manual_seed(100 + rank)  # different data per rank
        x = torch.randn(16, 3, 32, 32, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 10, (16,), generator=g).to(dev)

        def step():
            opt.zero_grad(set_to_none=True)
            loss = F.cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            return loss

        run = GraphedStep(step, warmup=3, capture_error_mode="thread_local")
        assert comm.choices, "the eager warm-up must have probed the payload size"
        calls = comm.one_shot_calls
        for it in range(10):
            run()
            torch.cuda.synchronize()
            for p in model.parameters():
                ref = p.detach().clone()
                dist.broadcast(ref, 0)
                assert torch.equal(ref, p.detach()), f"replay {it}: weights diverged across ranks"
        # replays do not pass through Python: the counter moved only in the eager warm-up
        assert comm.one_shot_calls == calls
        comm.check()
        dist.barrier()
        torch.cuda.synchronize()
    finally:
        set_default_comm(None)
        comm.close()


def test_xgmi_whole_step_graph_two_ranks():
    run_distributed(_xgmi_whole_step_graph_body, 2, timeout=300)


# The five BASELINE pipelines (BASELINE.json configs 2-5 + DGC): each one's W = 2 exchange captured
# in a whole-step HIP graph on the one-shot xGMI comm (gathers, the gather-reduce all-reduce of
# PowerSGD's P / Q and DGC's clipping norm, QSGD's one-shot all-to-all), replayed, and compared
# with an EAGER W = 2 run of the same steps through the gloo comm -- not only across ranks
# (an exchange wrong identically on every rank must fail here).
REHEARSAL = {
    "topk": {"compressor": "topk", "compress_ratio": 0.01, "memory": "residual", "communicator": "allgather"},
    "dgc": {"compressor": "dgc", "compress_ratio": 0.01, "memory": "dgc", "communicator": "allgather"},
    "powersgd": {"compressor": "powersgd", "compress_rank": 4, "memory": "powersgd", "communicator": "allreduce"},
    "efsignsgd": {"compressor": "efsignsgd", "lr": 0.1, "memory": "efsignsgd", "communicator": "allreduce"},
    "qsgd": {"compressor": "qsgd", "quantum_num": 127, "memory": "none", "communicator": "allreduce"},
}


def _mlp():
    import torch.nn as nn

    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(256, 512), nn.ReLU(), nn.Linear(512, 384), nn.ReLU(), nn.Linear(384, 10))


def _rehearsal_body(rank, world, name, replays):
    import torch.nn.functional as F

    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer, FusedSGD, broadcast_parameters
    from grace_amd.parallel.comm import TorchComm
    from grace_amd.parallel.graph import GraphedStep
    from grace_amd.parallel.xgmi import XgmiComm

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    comm = XgmiComm(TorchComm(), capacity_mb=8.0, select="size")
    params = dict(REHEARSAL[name], world_size=world)
    g = torch.Generator().manual_seed(100 + rank)  # different data per rank
    x = torch.randn(64, 256, generator=g).to(dev)
    y = torch.randint(0, 10, (64,), generator=g).to(dev)

    def build(c):
        model = _mlp().to(dev)
        broadcast_parameters(model.state_dict(), root_rank=0)
        grc = grace_from_params(params, comm=c)
        opt = DistributedOptimizer(FusedSGD(list(model.parameters()), lr=0.05, momentum=0.5), grc,
                                   named_parameters=list(model.named_parameters()), overlap=False)
        return model, opt

    def stepper(model, opt):
        def step():
            opt.zero_grad(set_to_none=True)
            loss = F.cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            return loss
        return step

    try:
        m1, o1 = build(comm)
        run = GraphedStep(stepper(m1, o1), warmup=3, capture_error_mode="thread_local")
        calls = comm.one_shot_calls
        assert calls > 0, "the eager warm-up must have used the one-shot comm"
        for _ in range(replays):
            run()
        torch.cuda.synchronize()
        assert comm.one_shot_calls == calls  # the replays ran without Python
        comm.check()
        m2, o2 = build(TorchComm())
        step2 = stepper(m2, o2)
        for _ in range(3 + replays):  # the warm-up steps are real steps too
            step2()
        torch.cuda.synchronize()
        for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
            ref = a.detach().clone()
            dist.broadcast(ref, 0)
            assert torch.equal(ref, a.detach()), f"{name}: {n} differs across ranks"
            if name == "powersgd":  # P / Q are float SUMS: gloo's ring vs the rank-ordered gather-reduce
                torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-7,
                                           msg=lambda m: f"{name}: {n} graphed != eager: {m}")
            else:  # gathered payloads decoded in rank order / integer sums: bit-identical
                assert torch.equal(a.detach(), b.detach()), \
                    f"{name}: {n} graphed one-shot exchange != eager gloo exchange (max diff {(a - b).abs().max():.3g})"
        dist.barrier()
        torch.cuda.synchronize()
    finally:
        comm.close()


@pytest.mark.parametrize("name", sorted(REHEARSAL))
def test_pipeline_whole_step_graph_two_ranks_matches_eager(name):
    run_distributed(_rehearsal_body, 2, name, 6, timeout=300)
