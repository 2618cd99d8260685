"""GPU: native RCCL runtime + DDP comm hook on one MI355X (runs before the graph tests: the
file name sorts first, and RCCL is initialised in a fresh process)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl_group():
    if not dist.is_initialized():
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(_free_port())
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    # no later module uses the group; tear it down so its watchdog thread (which queries the
    # events of RCCL work in flight) cannot race a later module's global-mode graph capture
    if dist.is_initialized():
        torch.cuda.synchronize()
        dist.destroy_process_group()


def test_rccl_cta_probe_single_rank(nccl_group):
    """RcclComm.tuned: one communicator per ncclConfig_t (minCTAs, maxCTAs) candidate, each timed
    on an all-reduce of the given size (MAX over ranks), the fastest kept and working (W = 1 runs
    the whole probe path; the choice itself only matters on the 8-GPU mesh)."""
    from grace_amd.parallel.native_comm import RcclComm

    cands = ((0, 0), (8, 8), (16, 32))
    c = RcclComm.tuned(1 << 20, candidates=cands, iters=2, inline=True)
    assert tuple(c.choice["ctas"]) in cands and c.ctas == tuple(c.choice["ctas"])
    assert set(c.choice["us"]) == {f"{a}/{b}" for a, b in cands} and c.choice["bytes"] == 1 << 20
    assert c.inline and c.verify()
    t = torch.arange(1000, dtype=torch.float32, device="cuda")
    c.all_reduce(t)
    torch.cuda.synchronize()
    torch.testing.assert_close(t, torch.arange(1000, dtype=torch.float32, device="cuda"))
    fixed = RcclComm.from_process_group(ctas=(4, 4))
    assert fixed._c.min_ctas == 4 and fixed._c.max_ctas == 4 and fixed.verify()


def _net():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(3, 16, 3, padding=1), nn.BatchNorm2d(16), nn.ReLU(), nn.AdaptiveAvgPool2d(1),
                         nn.Flatten(), nn.Linear(16, 10)).cuda()


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(8, 3, 16, 16, generator=g).cuda(), torch.randint(0, 10, (8,), generator=g).cuda()


def test_native_rccl_comm_single_rank(nccl_group):
    from grace_amd.parallel.native_comm import RcclComm

    c = RcclComm.from_process_group()
    t = torch.arange(10, dtype=torch.float32, device="cuda")
    w = c.all_reduce(t, async_op=True)
    w.wait()
    out = torch.empty(10, device="cuda")
    c.all_gather_into(out, t).wait()
    c.broadcast(t, 0).wait()
    torch.cuda.synchronize()
    torch.testing.assert_close(out, t)
    # all-to-all (send/recv group; the QSGD reduce-scatter wire format): identity at W = 1, int8
    codes = torch.arange(-64, 64, dtype=torch.int8, device="cuda")
    recv = torch.empty_like(codes)
    c.all_to_all(recv, codes, async_op=True).wait()
    torch.cuda.synchronize()
    assert torch.equal(recv, codes)
    assert c.world_size == 1
    c.check()


def test_native_rccl_self_check(nccl_group):
    """from_process_group runs the cross-rank self-check (all-reduce, all-gather, group) before
    returning; verify() can be re-run, inline or forked, and agrees over the torch group."""
    from grace_amd.parallel.native_comm import RcclComm

    for inline in (False, True):
        c = RcclComm.from_process_group(inline=inline)  # verify=True: raises on a bad runtime
        assert c.verify(timeout_s=30.0) is True


def test_native_rccl_concurrent_issue_threads(nccl_group):
    """Two threads issuing collectives on one RcclComm at once (the DDP hook on the autograd
    thread + a main-thread all-reduce): the per-call issue state keeps each call on its own
    stream and device guard; every result is exact."""
    import threading

    from grace_amd.parallel.native_comm import RcclComm

    c = RcclComm.from_process_group()
    errs = []

    def worker(seed):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for i in range(200):
                    t = torch.full((257,), float(seed * 1000 + i), device="cuda")
                    c.all_reduce(t, async_op=True).wait()
                    o = torch.empty(257, device="cuda")
                    c.all_gather_into(o, t, async_op=True).wait()
                    if not torch.equal(o, t):
                        errs.append((seed, i))
            s.synchronize()
        except Exception as e:  # pragma: no cover
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    torch.cuda.synchronize()
    assert not errs, errs[:4]
    c.check()


def test_native_comm_drives_grace(nccl_group):
    from grace_amd import grace_from_params
    from grace_amd.parallel.native_comm import RcclComm

    grc = grace_from_params({"compressor": "signsgd", "communicator": "allreduce"}, comm=RcclComm.from_process_group())
    g = torch.randn(1000, device="cuda")
    out = grc.step(g, "x")
    torch.testing.assert_close(out, torch.where(g >= 0, 1.0, -1.0))


def test_native_inline_comm_in_graph(nccl_group):
    """Inline mode: collectives on the caller's stream, so a whole training step with the RCCL
    all-gather inside is captured in one HIP graph without an event fork/join (bench.py's
    --comm native-inline); replays train exactly like the local (no-collective) comm."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.comm import LocalComm
    from grace_amd.parallel.graph import GraphedStep
    from grace_amd.parallel.native_comm import RcclComm

    c = RcclComm.from_process_group(inline=True)
    assert c.inline
    p = {"compressor": "topk", "compress_ratio": 0.1, "memory": "residual", "communicator": "allgather"}
    x, y = _data()
    models = []
    for comm in (LocalComm(), c):
        m = _net()
        o = DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.5),
                                 grace_from_params(p, comm=comm), named_parameters=m.named_parameters())

        def step():
            o.zero_grad()
            loss = F.cross_entropy(m(x), y)
            loss.backward()
            o.step()
            return loss

        run = GraphedStep(step, warmup=3)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        models.append(m)
    for a, b in zip(models[0].parameters(), models[1].parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    c.check()


def test_native_group_collectives(nccl_group):
    """RcclComm.group(): all-gathers and sum all-reduces in ONE ncclGroupStart/End (the path
    GroupedComm.flush takes for a step's buckets), forked and inline, also inside a HIP graph."""
    from grace_amd.parallel.comm import GroupedComm
    from grace_amd.parallel.native_comm import RcclComm

    for inline in (False, True):
        c = RcclComm.from_process_group(inline=inline)
        gc = GroupedComm(c)
        a = torch.arange(1000, dtype=torch.float32, device="cuda")
        b = torch.randn(333, device="cuda")
        oa = torch.empty(1000, device="cuda")
        ob = torch.empty(333, device="cuda")
        r = torch.full((77,), 3.0, device="cuda")
        ws = [gc.all_gather_into(oa, a, async_op=True), gc.all_reduce(r, async_op=True),
              gc.all_gather_into(ob, b, async_op=True)]
        assert gc.pending == 3
        gc.flush()
        assert gc.pending == 0
        for w in ws:
            w.wait()
        torch.cuda.synchronize()
        torch.testing.assert_close(oa, a)
        torch.testing.assert_close(ob, b)
        torch.testing.assert_close(r, torch.full((77,), 3.0, device="cuda"))
    # grouped collectives captured in a graph (inline comm, as under bench.py --graph full)
    c = RcclComm.from_process_group(inline=True)
    gc = GroupedComm(c)
    src = torch.randn(4096, device="cuda")
    out = torch.empty(4096, device="cuda")
    red = torch.zeros(64, device="cuda")

    def body():
        w1 = gc.all_gather_into(out, src, async_op=True)
        w2 = gc.all_reduce(red, async_op=True)
        gc.flush()
        w1.wait()
        w2.wait()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    src.normal_()
    g.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(out, src)
    c.check()


def test_engine_groups_bucket_collectives_in_graph(nccl_group):
    """DistributedOptimizer with several buckets and group_collectives=True on the inline native
    comm, whole step captured: trains exactly like the ungrouped local comm."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer
    from grace_amd.parallel.comm import LocalComm
    from grace_amd.parallel.graph import GraphedStep
    from grace_amd.parallel.native_comm import RcclComm

    c = RcclComm.from_process_group(inline=True)
    p = {"compressor": "topk", "compress_ratio": 0.1, "memory": "residual", "communicator": "allgather"}
    x, y = _data()
    models = []
    for comm, grp in ((LocalComm(), False), (c, True)):
        m = _net()
        o = DistributedOptimizer(torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.5),
                                 grace_from_params(p, comm=comm), named_parameters=m.named_parameters(),
                                 bucket_cap_mb=0.002, overlap=False, group_collectives=grp)
        assert o.engine.grouped == grp and len(o.engine.buckets) > 1

        def step():
            o.zero_grad()
            loss = F.cross_entropy(m(x), y)
            loss.backward()
            o.step()
            return loss

        run = GraphedStep(step, warmup=3)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        models.append(m)
    for a, b in zip(models[0].parameters(), models[1].parameters()):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    c.check()


def test_ddp_hook_gpu(nccl_group):
    from grace_amd import grace_from_params
    from grace_amd.parallel import GraceHookState, grace_comm_hook

    m = _net()
    ddp = nn.parallel.DistributedDataParallel(m, device_ids=[0])
    ddp.register_comm_hook(GraceHookState(grace_from_params({"compressor": "topk", "compress_ratio": 0.2,
                                                             "communicator": "allgather"})), grace_comm_hook)
    x, y = _data()
    F.cross_entropy(ddp(x), y).backward()
    torch.cuda.synchronize()
    for prm in m.parameters():
        frac = (prm.grad != 0).float().mean().item()
        assert frac <= 0.2 + 1.0 / prm.numel() + 1e-6


def _split_net(seed=0):
    from grace_amd.ops.wgrad import Conv2dSplitGrad

    torch.manual_seed(seed)
    return nn.Sequential(Conv2dSplitGrad(3, 32, 3, padding=1, bias=False), nn.ReLU(),
                         Conv2dSplitGrad(32, 32, 3, stride=2, padding=1, bias=False), nn.ReLU(),
                         nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(32, 10)).cuda()


@pytest.fixture
def side_delay(request):
    """Race detector: every side-stream fork first spins ~0.1 ms (ops/wgrad.py _SIDE_DELAY), so a
    consumer that reads a side-stream weight gradient without joining reads a stale one."""
    from grace_amd.ops import wgrad as _wg

    old = _wg._SIDE_DELAY
    _wg._SIDE_DELAY = getattr(request, "param", 0)
    yield _wg._SIDE_DELAY
    _wg._SIDE_DELAY = old


@pytest.mark.parametrize("side_delay", [0, 200000], indirect=True)
@pytest.mark.parametrize("defer", [False, True])
def test_ddp_hook_split_grad_convs_match_plain_model(nccl_group, defer, side_delay):
    """DDP + hook over split-gradient convs (ops/wgrad.py).  Immediate hook: the reducer reads
    gradients mid-backward, so DDP-managed weights compute their gradients in line, and
    (gradient_as_bucket_view) straight into the bucket once the hook has seen it.  Deferred hook
    (GraceHookState(defer=True)): weight gradients run on the side stream, written INTO the bucket
    views (library kernels included), and flush() joins before the exchange.  Either way the
    gradients equal a plain model's, every step."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import GraceHookState, grace_comm_hook

    m, ref = _split_net(), _split_net()
    ddp = nn.parallel.DistributedDataParallel(m, device_ids=[0], gradient_as_bucket_view=True,
                                              broadcast_buffers=False)
    st = GraceHookState(grace_from_params({"compressor": "none", "communicator": "allreduce"}), model=ddp,
                        defer=defer)
    ddp.register_comm_hook(st, grace_comm_hook)
    g = torch.Generator().manual_seed(3)
    for step in range(6):
        x = torch.randn(16, 3, 24, 24, generator=g).cuda()
        y = torch.randint(0, 10, (16,), generator=g).cuda()
        for p in list(m.parameters()) + list(ref.parameters()):
            p.grad = None
        F.cross_entropy(ddp(x), y).backward()
        st.flush()
        F.cross_entropy(ref(x), y).backward()
        torch.cuda.synchronize()
        for a, b in zip(m.parameters(), ref.parameters()):
            assert a._grace_ddp
            tol = 1e-4 * float(b.grad.abs().max()) + 1e-6
            assert float((a.grad - b.grad).abs().max()) <= tol, step
    conv_w = [mod.weight for mod in m if hasattr(mod, "kernel_size")]
    for w in conv_w:  # the gradient IS the bucket view the hook marked (no reducer copy)
        assert w._grace_grad_view.data_ptr() == w.grad.data_ptr()


@pytest.mark.parametrize("side_delay", [0, 200000], indirect=True)
@pytest.mark.parametrize("mode", ["immediate", "deferred", "deferred-split"])
def test_ddp_hook_graph_capture(nccl_group, mode, side_delay):
    """A whole DDP step (forward, backward with the comm hook, optimizer) captured in a HIP graph:
    DDP is built under the capture stream (its AccumulateGrad nodes run there) and warmed up past
    its runtime-logging iterations; replays equal the same steps run eagerly.  ``deferred``: the
    hook queues the buckets and GraceDDPOptimizer.step() flushes them (weight gradients forked
    onto the side stream); ``deferred-split``: that step captured as split graphs."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import GraceDDPOptimizer, GraceHookState, grace_comm_hook
    from grace_amd.parallel.graph import GraphedStep

    g = torch.Generator().manual_seed(5)
    x = torch.randn(16, 3, 24, 24, generator=g).cuda()
    y = torch.randint(0, 10, (16,), generator=g).cuda()
    finals = []
    for graphed in (False, True):
        m = _split_net(seed=1)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            ddp = nn.parallel.DistributedDataParallel(m, device_ids=[0], gradient_as_bucket_view=True,
                                                      broadcast_buffers=False)
        st = GraceHookState(grace_from_params({"compressor": "none", "communicator": "allreduce"}), model=ddp,
                            defer=mode != "immediate")
        ddp.register_comm_hook(st, grace_comm_hook)
        opt = GraceDDPOptimizer(torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.5), st)

        def step():
            opt.zero_grad(set_to_none=True)
            loss = F.cross_entropy(ddp(x), y)
            loss.backward()
            opt.step()
            return loss

        if graphed:
            # DDP logs runtime stats in its first 10 steps
            run = GraphedStep(step, warmup=11, stream=s, split=mode == "deferred-split")
            if mode == "deferred-split":
                assert run.g_side is not None and run.g_a2 is not None
            for _ in range(4):
                run()
        else:
            with torch.cuda.stream(s):
                for _ in range(11 + 4):  # the warm-up steps + 4 replays (capture itself runs nothing)
                    step()
        torch.cuda.synchronize()
        finals.append([p.detach().clone() for p in m.parameters()])
    for i, (a, b) in enumerate(zip(*finals)):
        err = float((a - b).abs().max())
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5,
                                   msg=f"{mode}: parameter {i} {tuple(a.shape)} max abs err {err:.3g}")


def _masked_reference(recorded):
    """A bn_act for the float64 CPU reference that applies the GPU run's ReLU decisions: y =
    (bn(x) + residual) * M_gpu, so the reference differentiates the SAME piecewise-linear function
    the GPU run did.  (A ReLU input within fp32 rounding of 0 legitimately flips between two fp32
    runs that sum in different orders -- and then that one element's gradient, |dy| there, shows up
    in every BN bias / conv weight gradient below it: that, not a race, was the r4 "intermittent
    plain-DDP mismatch", one flipped bit of 32768 in layer3.0.bn2, tools/gpu/bn_bwd_capture.py.)"""
    import torch.nn as nn

    it = iter(recorded)

    def bn_act(x, bn, residual=None, relu=False, dual=False, **_):
        y = nn.BatchNorm2d.forward(bn, x)
        if residual is not None:
            y = y + residual
        if relu:
            y = y * next(it).to(y.dtype)
        return (y, y) if dual else y
    return bn_act


def _record_masks(store):
    from grace_amd.ops import bnact

    real = bnact.bn_act

    def bn_act(x, bn, residual=None, relu=False, dual=False, *a, **k):
        out = real(x, bn, residual, relu, dual, *a, **k)
        if relu:
            y = out[0] if isinstance(out, tuple) else out
            store.append((y.detach() > 0).cpu())
        return out
    return bn_act


@pytest.fixture(params=[None, "mfma_t2"], ids=["autotuned", "forced-dgrad-mfma_t2"])
def dgrad_choice(request):
    """The second case pins every 3x3 data gradient to the 128x64 MFMA tile: the configuration
    that flipped layer3.0.bn2's ReLU bit in (almost) every process with the r4 GPU-vs-GPU test."""
    from grace_amd.ops import conv

    if request.param is None:
        yield None
        return
    real = conv._pick3
    conv._pick3 = lambda d, x, w, dy, s: (request.param if d == "dgrad" and s == 1 and w.shape[2] == 3
                                          else real(d, x, w, dy, s))
    try:
        yield request.param
    finally:
        conv._pick3 = real


def test_plain_ddp_resnet_grads_match_fp64(nccl_group, dgrad_choice):
    """grace_amd.models.resnet under PLAIN DDP (no GRACE hook, no engine): its parameters are not
    tagged joinable, so every weight gradient is computed in line and the reducer's mid-backward
    reads see finished gradients.  Both the side-stream-switch-off and -on runs are compared with
    a float64 CPU reference of the same weights and input that takes each run's ReLU decisions
    (``_masked_reference``); the tolerance is fp32 summation over the reductions feeding each
    gradient (<= 4096 terms: 2e-4 of the tensor's max).  A race -- a gradient read before its
    producer finished -- would be off by O(1), not by rounding (ADVICE r3 high / VERDICT r4 #1)."""
    import copy

    from grace_amd.models import resnet18_cifar
    from grace_amd.ops import bnact, bnconv, wgrad

    torch.manual_seed(0)
    base = resnet18_cifar()  # CPU fp32: the source of both the GPU runs and the fp64 reference
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8, 3, 16, 16, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    names = [n for n, _ in base.named_parameters()]
    real = bnact.bn_act
    for stream_on in (False, True):
        masks = []
        m = copy.deepcopy(base).cuda().to(memory_format=torch.channels_last)
        ddp = nn.parallel.DistributedDataParallel(m, device_ids=[0], broadcast_buffers=False)
        wgrad.set_enabled(stream_on)
        try:
            for it in range(2):
                for p in m.parameters():
                    p.grad = None
                masks.clear()
                if it == 1:
                    bnact.bn_act = bnconv.bn_act = _record_masks(masks)
                try:
                    F.cross_entropy(ddp(x.cuda().contiguous(memory_format=torch.channels_last)), y.cuda()).backward()
                finally:
                    bnact.bn_act = bnconv.bn_act = real
        finally:
            wgrad.set_enabled(True)
        assert not any(wgrad.joinable(p) for p in m.parameters())
        torch.cuda.synchronize()
        got = [p.grad.detach().double().cpu() for p in m.parameters()]
        ref_m = copy.deepcopy(base).double()
        bnact.bn_act = bnconv.bn_act = _masked_reference(masks)
        try:
            F.cross_entropy(ref_m(x.double()), y).backward()
        finally:
            bnact.bn_act = bnconv.bn_act = real
        bad = []
        for n, a, p in zip(names, got, ref_m.parameters()):
            b = p.grad
            err, tol = float((a - b).abs().max()), 2e-4 * float(b.abs().max()) + 1e-9
            if err > tol:
                bad.append(f"{n}{tuple(a.shape)}: {err:.3g} > {tol:.3g}")
        assert not bad, f"stream {'on' if stream_on else 'off'}: {len(bad)} of {len(names)} differ from fp64, " \
                        "deepest first: " + "; ".join(bad[::-1])
