"""GPU: weight gradients on the side stream (grace_amd/ops/wgrad.py) give the same gradients as the
in-line backward -- eagerly, through the GRACE engine's bucket gather, and inside a captured
whole-step HIP graph (the fork is a parallel graph branch)."""
import os
import pytest
import torch
import torch.nn.functional as F

from grace_amd.ops import wgrad
from grace_amd.ops.wgrad import Conv2dSplitGrad

pytestmark = pytest.mark.gpu


def _close(a, b, msg=None):
    """fp32 agreement up to summation order (MIOpen's weight-gradient solvers accumulate with
    atomics: run-to-run differences ~1e-6 of the tensor's scale)"""
    a, b = a.detach(), b.detach()
    atol = 1e-4 * float(b.abs().max()) + 1e-7
    err = float((a.double() - b.double()).abs().max())
    torch.testing.assert_close(a, b, rtol=1e-4, atol=atol,
                               msg=f"{msg}: max abs err {err:.3g} (atol {atol:.3g}, max |ref| {float(b.abs().max()):.3g})")


@pytest.fixture
def bn_deterministic():
    """fixed-order BN backward reductions: eager and replayed steps then differ only by MIOpen's
    atomic weight gradients (the default atomic BN totals add order noise that a few SGD steps
    amplify in cancellation-heavy sums such as a BN bias gradient)"""
    from grace_amd.ops import _native

    _native.lib().bn_set_deterministic(True)
    yield
    _native.lib().bn_set_deterministic(os.environ.get("GRACE_BN_DETERMINISTIC") == "1")


def _grads(model, x, y):
    for p in model.parameters():
        p.grad = None
    loss = F.cross_entropy(model(x), y)
    loss.backward()
    return [p.grad.detach().clone() for p in model.parameters()]


@pytest.mark.parametrize("stride,pad,k", [(1, 1, 3), (2, 1, 3), (2, 0, 1), (2, 3, 7)])
def test_split_conv_matches_conv2d(stride, pad, k):
    torch.manual_seed(0)
    conv = Conv2dSplitGrad(16, 32, k, stride=stride, padding=pad, bias=False).cuda()
    ref = torch.nn.Conv2d(16, 32, k, stride=stride, padding=pad, bias=False).cuda()
    ref.load_state_dict(conv.state_dict())
    x = torch.randn(4, 16, 20, 20, device="cuda").contiguous(memory_format=torch.channels_last)
    wgrad.mark_joinable(conv.parameters())  # fork: the final callback joins before the compare
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = conv(xa), ref(xb)
    dy = torch.randn_like(ya)
    ya.backward(dy)
    yb.backward(dy)
    torch.testing.assert_close(ya, yb, rtol=0, atol=0)
    _close(xa.grad, xb.grad)
    _close(conv.weight.grad, ref.weight.grad)


def _small_cnn(num_classes=10):
    """conv3x3 -> BN+ReLU -> strided conv3x3 -> BN+ReLU -> 1x1 (Conv1x1F32) -> BN+ReLU -> pool -> fc:
    every conv flavour of the ResNets, shallow enough that fp32 run-to-run differences (MIOpen's
    atomic solvers) stay ~1e-6 (a deep ResNet at batch 4 amplifies them to percent level through
    its small-sample BN statistics, with or without the side stream)."""
    from grace_amd.ops.bnact import BatchNormAct2d
    from grace_amd.ops.conv import Conv1x1F32
    from grace_amd.ops.pool import GlobalAvgPoolFlat

    return torch.nn.Sequential(
        Conv2dSplitGrad(3, 32, 3, padding=1, bias=False), BatchNormAct2d(32, relu=True),
        Conv2dSplitGrad(32, 64, 3, stride=2, padding=1, bias=False), BatchNormAct2d(64, relu=True),
        Conv1x1F32(64, 128), BatchNormAct2d(128, relu=True),
        GlobalAvgPoolFlat(), torch.nn.Linear(128, num_classes))


def test_side_stream_grads_equal_inline():
    torch.manual_seed(0)
    model = _small_cnn().cuda().to(memory_format=torch.channels_last)
    wgrad.mark_joinable(model.parameters())  # backward's final callback joins before _grads clones
    x = torch.randn(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")
    wgrad.set_enabled(False)
    try:
        _grads(model, x, y)  # settle autotuned choices (same backend both runs)
        ref = _grads(model, x, y)
    finally:
        wgrad.set_enabled(True)
    for _ in range(3):
        got = _grads(model, x, y)  # no host sync between backward and the clone: the joins order it
        for (n, _), a, b in zip(model.named_parameters(), got, ref):
            _close(a, b, msg=n)


@pytest.mark.parametrize("tail", [False, True])
@pytest.mark.parametrize("delay", [0, 200000])
@pytest.mark.parametrize("split", [False, True])
def test_engine_graph_with_side_stream_wgrad(bn_deterministic, split, delay, tail, monkeypatch):
    """an engine step captured in a whole-step graph with the wgrad forks (parallel graph
    branches, joined before the bucket gather) matches the eager steps (parameters after 4 steps);
    split=True: captured as two linear graphs (critical / side stream) joined by flag words plus
    the post-join graph (parallel/graph.py GraphedStep split); delay > 0: the race detector (every
    fork spins first on the side stream, so a missing join reads stale gradients)"""
    monkeypatch.setattr(wgrad, "_SIDE_DELAY", delay)
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer, FusedSGD
    from grace_amd.parallel.graph import GraphedStep

    def build():
        torch.manual_seed(1)
        m = _small_cnn().cuda().to(memory_format=torch.channels_last)
        grc = grace_from_params({"compressor": "none", "memory": "none", "communicator": "allreduce",
                                 "world_size": 1})
        opt = DistributedOptimizer(FusedSGD(list(m.parameters()), lr=0.05, momentum=0.5), grc,
                                   named_parameters=list(m.named_parameters()), overlap=False, tail_bucket=tail)
        if tail:  # the first conv's weight alone in the last bucket
            assert len(opt.engine.buckets) == 2 and len(opt.engine.buckets[-1].params) == 1
        return m, opt

    x = torch.randn(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")

    def make_step(m, opt):
        def step():
            opt.zero_grad(set_to_none=True)
            loss = F.cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            return loss
        return step

    m1, o1 = build()
    s1 = make_step(m1, o1)
    for _ in range(7):
        s1()
    m2, o2 = build()
    g = GraphedStep(make_step(m2, o2), warmup=3, split=split)  # 3 eager warm-up steps + capture (not a step)
    if split:
        assert g.g_side is not None and g.g_a2 is not None and len(g._sc.events) >= 3
    for _ in range(4):
        g()
    torch.cuda.synchronize()
    # parameters after 7 SGD steps: fp32 order noise of MIOpen's / the split-K GEMM's atomic weight
    # gradients (~1e-7 relative per step) grows in cancellation-heavy sums (a BN bias gradient is a
    # sum of +-terms ~1e3 x its value); a missing join would corrupt whole tensors at the 1e-2 level
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        err = float((a - b).abs().max())
        assert err <= 1e-3 * float(b.abs().max()) + 2e-5, f"{n}: max abs err {err:.3g}"


@pytest.mark.parametrize("split", [False, True])
def test_topk_graph_with_side_stream_runs(split):
    """ResNet-50 Top-K 1 % whole-step graph with the wgrad forks: replays are finite and the
    exchange leaves ~1 % non-zero gradients (one forked graph, or the split A / B / A2 graphs)"""
    from grace_amd import grace_from_params
    from grace_amd.models import resnet50
    from grace_amd.parallel import DistributedOptimizer, FusedSGD
    from grace_amd.parallel.graph import GraphedStep

    torch.manual_seed(1)
    m = resnet50(num_classes=10).cuda().to(memory_format=torch.channels_last)
    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.01, "memory": "residual",
                             "communicator": "allgather", "world_size": 1})
    opt = DistributedOptimizer(FusedSGD(list(m.parameters()), lr=0.01, momentum=0.5), grc,
                               named_parameters=list(m.named_parameters()), overlap=False)
    x = torch.randn(8, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device="cuda")

    def step():
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(m(x), y)
        loss.backward()
        opt.step()
        return loss

    g = GraphedStep(step, warmup=3, split=split)
    for _ in range(3):
        loss = g()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item()
    nz = sum(int((p.grad != 0).sum()) for p in m.parameters())
    total = sum(p.numel() for p in m.parameters())
    assert 0 < nz <= 0.02 * total


@pytest.mark.parametrize("k,pad", [(3, 1), (3, 0), (5, 2), (1, 0)])
def test_dgrad_forms_agree(k, pad):
    """the flipped-filter forward form of a stride-1 data gradient equals the backward-data solver"""
    torch.manual_seed(0)
    x = torch.randn(2, 24, 15, 13, device="cuda").contiguous(memory_format=torch.channels_last)
    w = torch.randn(40, 24, k, k, device="cuda").contiguous(memory_format=torch.channels_last)
    dy = torch.randn(2, 40, 15 + 2 * pad - k + 1, 13 + 2 * pad - k + 1, device="cuda").contiguous(
        memory_format=torch.channels_last)
    ref = torch.ops.aten.convolution_backward(dy.double(), x.double(), w.double(), None, [1, 1], [pad, pad], [1, 1],
                                              False, [0, 0], 1, [True, False, False])[0]
    fwd = F.conv2d(dy, wgrad._flipped(w), None, 1, [k - 1 - pad, k - 1 - pad])
    _close(fwd.double(), ref)
    wgrad._DG_CHOICE.clear()
    auto = wgrad._DG_AUTO
    wgrad._DG_AUTO = True
    try:
        got = wgrad._dgrad(dy, x, w, [1, 1], [pad, pad], [1, 1], 1)
    finally:
        wgrad._DG_AUTO = auto
    _close(got.double(), ref)


def test_untagged_parameters_stay_in_line():
    """a model whose gradients nobody joins (no GRACE engine: plain DDP, hooks, user code) never
    forks a weight gradient, so a post-accumulate-grad hook reading .grad mid-backward on the
    compute stream sees the finished gradient (side-stream race)"""
    torch.manual_seed(0)
    model = _small_cnn().cuda().to(memory_format=torch.channels_last)
    x = torch.randn(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")
    wgrad.set_enabled(False)
    try:
        _grads(model, x, y)
        ref = _grads(model, x, y)
    finally:
        wgrad.set_enabled(True)
    seen = {}
    hooks = [p.register_post_accumulate_grad_hook(lambda p: seen.__setitem__(id(p), p.grad.clone()))
             for p in model.parameters()]
    try:
        for _ in range(2):
            seen.clear()
            got = _grads(model, x, y)
            assert not wgrad._pending.get(torch.cuda.current_device())
            for (n, p), a, b in zip(model.named_parameters(), got, ref):
                _close(a, b, msg=n)
                _close(seen[id(p)], b, msg=f"hook {n}")  # the clone ran mid-backward
    finally:
        for h in hooks:
            h.remove()


def test_second_capture_after_eager_steps(bn_deterministic):
    """bench.py's sequence: a captured engine step, eager (profiled) steps whose last loss stays
    referenced, then a second engine captured for the no-op split.  The eager steps' autograd
    graph must be released before the second capture (bench.py drops it) -- kept alive it binds the
    parameters' AccumulateGrad nodes to the eager stream and the capture fails with unjoined work."""
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer, FusedSGD
    from grace_amd.parallel.comm import LocalComm
    from grace_amd.parallel.graph import GraphedStep

    torch.manual_seed(2)
    m = _small_cnn().cuda().to(memory_format=torch.channels_last)
    x = torch.randn(16, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (16,), device="cuda")
    base = FusedSGD(list(m.parameters()), lr=0.05, momentum=0.5)

    def make(opt):
        def step():
            opt.zero_grad(set_to_none=True)
            loss = F.cross_entropy(m(x), y)
            loss.backward()
            opt.step()
            return loss
        return step

    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.05, "memory": "residual",
                             "communicator": "allgather", "world_size": 1})
    o1 = DistributedOptimizer(base, grc, named_parameters=list(m.named_parameters()), overlap=False)
    g1 = GraphedStep(make(o1), warmup=3)
    for _ in range(2):
        g1()
    for _ in range(2):  # eager steps, as bench.py's exposed-exchange split
        o1.zero_grad(set_to_none=True)
        l2 = F.cross_entropy(m(x), y)
        l2.backward()
        o1.step()
    l2 = None  # noqa: F841  (bench.py releases it the same way)
    o1.engine.remove()
    o2 = DistributedOptimizer(base, grace_from_params({"compressor": "none", "communicator": "allreduce"},
                                                      comm=LocalComm()),
                              named_parameters=list(m.named_parameters()), overlap=False)
    g2 = GraphedStep(make(o2), warmup=3)
    for _ in range(2):
        loss = g2()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item()


