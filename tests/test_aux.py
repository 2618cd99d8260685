"""Auxiliary subsystems: checkpoint/resume of GRACE state, fault injection, watchdog, profiler."""
import os
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(10, 32), nn.ReLU(), nn.Linear(32, 3))


def _train(model, opt, steps, seed0):
    for s in range(steps):
        g = torch.Generator().manual_seed(seed0 + s)
        x, y = torch.randn(8, 10, generator=g), torch.randint(0, 3, (8,), generator=g)
        opt.zero_grad()
        F.cross_entropy(model(x), y).backward()
        opt.step()


def test_checkpoint_resume_preserves_grace_state(tmp_path):
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.utils import checkpoint

    params = {"compressor": "signum", "momentum": 0.9, "memory": "residual", "communicator": "allgather"}

    def make():
        m = _model()
        return m, DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9),
                                       grace_from_params(params), named_parameters=m.named_parameters())

    m1, o1 = make()
    _train(m1, o1, 3, 0)
    path = str(tmp_path / "ck.pt")
    checkpoint.save(path, m1, o1)
    _train(m1, o1, 2, 100)  # continue the original

    m2, o2 = make()
    checkpoint.load(path, m2, o2)
    _train(m2, o2, 2, 100)  # resume
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b)


def _ckpt_w2_body(rank, world, path):
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.utils import checkpoint

    params = {"compressor": "topk", "compress_ratio": 0.2, "memory": "residual", "communicator": "allgather",
              "world_size": world}

    def make():
        m = _model()
        return m, DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9),
                                       grace_from_params(params), named_parameters=m.named_parameters())

    m1, o1 = make()
    _train(m1, o1, 3, 10 * rank)  # rank-specific data: rank-specific residuals
    res1 = {k: v.clone() for k, v in o1.engine.grc.memory.residuals.items()}
    checkpoint.save(path, m1, o1)  # per-rank GRACE state by default at W > 1
    assert os.path.exists(checkpoint.grace_path(path, rank))
    m2, o2 = make()
    checkpoint.load(path, m2, o2)
    res2 = o2.engine.grc.memory.residuals
    assert res1.keys() == res2.keys()
    for k in res1:
        assert torch.equal(res1[k], res2[k]), "rank got back another rank's residual"
    # residuals really differ across ranks (else the test proves nothing)
    k0 = sorted(res1)[0]
    out = [torch.empty_like(res1[k0]) for _ in range(world)]
    dist.all_gather(out, res1[k0].contiguous())
    assert not torch.equal(out[0], out[1])
    _train(m1, o1, 2, 100 + rank)
    _train(m2, o2, 2, 100 + rank)
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b)


def test_checkpoint_per_rank_grace_state_w2(tmp_path):
    run_distributed(_ckpt_w2_body, 2, str(tmp_path / "ck.pt"))


def test_checkpoint_bf16_masters_roundtrip(tmp_path):
    """BF16Weights: the fp32 masters (not the bf16 working copies) are saved and restored."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.precision import BF16Weights
    from grace_amd.utils import checkpoint

    def make():
        m = _model()
        w = BF16Weights(m)
        o = DistributedOptimizer(torch.optim.SGD(list(w.master_parameters(m)), lr=0.1, momentum=0.9),
                                 grace_from_params({"compressor": "none", "communicator": "allreduce"}),
                                 named_parameters=list(w.named_master_parameters(m)), weights=w)
        return m, w, o

    def train(m, o, steps, seed0):
        for s in range(steps):
            g = torch.Generator().manual_seed(seed0 + s)
            x, y = torch.randn(8, 10, generator=g), torch.randint(0, 3, (8,), generator=g)
            o.zero_grad()
            with torch.autocast("cpu", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x), y)
            loss.backward()
            o.step()

    m1, w1, o1 = make()
    train(m1, o1, 3, 0)
    path = str(tmp_path / "ck.pt")
    checkpoint.save(path, m1, o1, weights=w1)
    m2, w2, o2 = make()
    checkpoint.load(path, m2, o2, weights=w2)
    for a, b in zip(w1.masters, w2.masters):
        assert a.dtype == torch.float32 and torch.equal(a, b)
    for a, b in zip(w1.working, w2.working):
        assert torch.equal(a, b)
    train(m1, o1, 2, 50)
    train(m2, o2, 2, 50)
    for a, b in zip(w1.masters, w2.masters):
        torch.testing.assert_close(a, b)


def test_checkpoint_loader_is_weights_only(tmp_path):
    from grace_amd.utils import checkpoint

    m = _model()
    path = str(tmp_path / "m.pt")
    checkpoint.save(path, m, extra={"epoch": 3})
    assert checkpoint.load(path, _model()) == {"epoch": 3}


def test_profiler_cpu_noop():
    from grace_amd import grace_from_params
    from grace_amd.utils.profiler import GraceProfiler

    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.1, "communicator": "allgather"})
    grc.profiler = GraceProfiler()
    grc.step(torch.randn(100), "x")
    grc.profiler.step()
    rep = grc.profiler.report()
    assert rep["bytes_per_step"] == 8 * 10  # 10 values (fp32) + 10 indices (int32)


def test_watchdog_times_out():
    from grace_amd.parallel.launch import Watchdog

    class Never:
        def is_completed(self):
            return False

    class Aborter:
        aborted = False

        def abort(self):
            Aborter.aborted = True

    wd = Watchdog(timeout_s=0.2, poll_s=0.05, abort=Aborter())
    wd.track(Never(), "stuck all_gather")
    time.sleep(0.6)
    with pytest.raises(TimeoutError):
        wd.check()
    assert Aborter.aborted
    wd.close()


def _fault_body(rank, world, marker):
    from grace_amd import grace_from_params

    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.1, "communicator": "allgather",
                             "world_size": world})
    grc.step(torch.randn(1000), "w")  # healthy step
    dist.barrier()
    if rank == 1:
        os._exit(0)  # injected failure: the peer disappears mid-training
    try:
        for _ in range(5):
            grc.step(torch.randn(1000), "w")
    except Exception as e:  # clean error instead of a hang
        with open(marker, "w") as f:
            f.write(repr(e))
        os._exit(0)
    os._exit(3)


def test_fault_injection_peer_death(tmp_path):
    marker = str(tmp_path / "caught")
    try:
        run_distributed(_fault_body, 2, marker, timeout=120)
    except AssertionError:
        pass
    assert os.path.exists(marker), "surviving rank did not observe the failure"


def test_packing_helpers_roundtrip_and_reference_format():
    from grace_amd.ops import packing as P

    for n in (1, 3, 4, 5, 8, 1001):
        a = torch.randint(0, 4, (n,), generator=torch.Generator().manual_seed(n))
        assert torch.equal(P.decode_byte(P.encode_byte(a), n), a.to(torch.int32))
        assert torch.equal(P.unpack2(P.pack2(a), n), a.to(torch.int32))
    # reference layout: quarters (n=4 pads 4 more entries 0..3 -> 2 bytes)
    enc = P.encode_byte(torch.tensor([1, 2, 3, 0]))
    assert enc.tolist() == [1 + 4 * 3 + 16 * 0 + 64 * 2, 2 + 4 * 0 + 16 * 1 + 64 * 3]


def test_profiler_splits_comm_and_decompress():
    """GraceProfiler phases: compress / comm / decompress are separate entries (bench.py reports
    them as the exchange split); CPU: events are no-ops, bytes are still counted."""
    from grace_amd import grace_from_params
    from grace_amd.utils.profiler import GraceProfiler

    grc = grace_from_params({"compressor": "fp16", "communicator": "allreduce"})
    grc.profiler = GraceProfiler()
    h, ctx = grc.send_step(torch.randn(256), "x")
    out = grc.receive_step(h, ctx)
    grc.profiler.step()
    assert out.shape == (256,)
    assert grc.profiler.report()["bytes_per_step"] == 512


def test_engine_watchdog_raises_in_training_thread():
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.launch import Watchdog

    m = _model()
    wd = Watchdog(timeout_s=60, poll_s=0.05)
    o = DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1), grace_from_params({"compressor": "none"}),
                             named_parameters=m.named_parameters(), watchdog=wd)
    _train(m, o, 1, 0)  # healthy
    wd._failure = "all_gather of bucket 0 did not complete within 60s"  # injected
    with pytest.raises(TimeoutError):
        _train(m, o, 1, 1)
    wd.close()


def test_native_library_loads_on_cpu_host():
    """The built extension imports on the host (no GPU needed for the module itself)."""
    from grace_amd.ops import _native

    if not os.path.exists(os.path.join(os.path.dirname(os.path.dirname(__file__)), "grace_amd", "_C.so")):
        pytest.skip("extension not built")
    assert _native.available(), _native._err
    assert "gfx950" in _native.lib().build_info()


def _capture_mode_rank(rank, world):
    from grace_amd.parallel.graph import _nccl_group_up

    assert dist.is_initialized() and dist.get_backend() == "gloo"
    assert not _nccl_group_up()  # gloo has no watchdog querying HIP events: global capture is fine


def test_graphed_step_capture_mode_follows_the_process_group():
    """GraphedStep(capture_error_mode=None) captures thread-locally only under an RCCL ("nccl")
    group, whose watchdog thread queries HIP events while the training thread captures."""
    from grace_amd.parallel.graph import _nccl_group_up

    assert not dist.is_initialized() and not _nccl_group_up()
    run_distributed(_capture_mode_rank, 1)


def test_rccl_backend_string_forms():
    """Backend strings that include RCCL in any form select the thread-local capture."""
    from grace_amd.parallel.graph import _is_rccl_backend

    assert _is_rccl_backend("nccl") and _is_rccl_backend("cpu:gloo,cuda:nccl")
    assert _is_rccl_backend("cuda:nccl") and not _is_rccl_backend("gloo") and not _is_rccl_backend(None)


def _capture_mode_mixed_rank(rank, world):
    import torch.distributed.distributed_c10d as c10d

    from grace_amd.parallel import graph as G
    from grace_amd.parallel import native_comm

    real = dist.get_backend
    assert not G._nccl_group_up()
    # 1. the default group created without a backend on a GPU box reports a mixed string
    dist.get_backend = lambda g=None: "cpu:gloo,cuda:nccl" if g is None else real(g)
    c10d.get_backend = dist.get_backend
    try:
        assert G._nccl_group_up()
    finally:
        dist.get_backend = c10d.get_backend = real
    # 2. an NCCL SUBGROUP over a gloo default group (the step's own group is what matters)
    sub = dist.new_group(ranks=list(range(world)), backend="gloo")
    dist.get_backend = lambda g=None: "nccl" if g is sub else real(g)
    c10d.get_backend = dist.get_backend
    try:
        assert G._nccl_group_up()
    finally:
        dist.get_backend = c10d.get_backend = real
    assert not G._nccl_group_up()
    # 3. a live native RCCL communicator (its proxy thread makes HIP calls) also counts
    orig = native_comm.live_count
    native_comm.live_count = lambda: 1
    try:
        assert G._nccl_group_up()
    finally:
        native_comm.live_count = orig


def test_capture_mode_sees_mixed_backends_and_subgroups():
    run_distributed(_capture_mode_mixed_rank, 2)
