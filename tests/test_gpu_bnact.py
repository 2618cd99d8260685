"""Fused BN(+residual)(+ReLU) HIP kernels (csrc/kernels/bnact.hip) vs a plain PyTorch fp32
reference of the same op."""
import os
import pytest
import torch
import torch.nn.functional as F

from grace_amd.ops import _native
from grace_amd.ops.bnact import BatchNormAct2d, _fusable

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(n, c, h, w, relu, with_res, seed=0, dtype=torch.bfloat16):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = (torch.randn(n, c, h, w, generator=g) * 2 + 0.5).to(DEV, dtype)
    x = x.contiguous(memory_format=torch.channels_last)
    res = None
    if with_res:
        res = torch.randn(n, c, h, w, generator=g).to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, c, h, w, generator=g).to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    m = BatchNormAct2d(c, relu=relu).to(DEV)
    with torch.no_grad():
        m.weight.copy_(torch.rand(c, generator=g) + 0.5)
        m.bias.copy_(torch.randn(c, generator=g) * 0.1)
    return m, x, res, dy


def _reference(m, x, res, dy, relu):
    xf = x.detach().float().requires_grad_(True)
    rf = res.detach().float().requires_grad_(True) if res is not None else None
    w = m.weight.detach().clone().requires_grad_(True)
    b = m.bias.detach().clone().requires_grad_(True)
    rm = torch.zeros_like(m.running_mean)
    rv = torch.ones_like(m.running_var)
    y = F.batch_norm(xf, rm, rv, w, b, True, m.momentum, m.eps)
    if rf is not None:
        y = y + rf
    if relu:
        y = F.relu(y)
    y.backward(dy.float())
    return y.detach(), xf.grad, (rf.grad if rf is not None else None), w.grad, b.grad, rm, rv


@pytest.mark.parametrize("shape", [(4, 64, 9, 9), (2, 256, 7, 5), (3, 2048, 3, 3), (1, 8, 2, 3), (8, 96, 4, 4),
                                   (32, 128, 28, 28), (32, 1024, 14, 14), (16, 512, 17, 3), (32, 64, 112, 112),
                                   (32, 64, 56, 56), (32, 2048, 7, 7), (31, 512, 14, 13)])
@pytest.mark.parametrize("relu,with_res", [(False, False), (True, False), (True, True), (False, True)])
def test_bnact_matches_fp32_reference(shape, relu, with_res):
    assert _native.available()
    m, x, res, dy = _case(*shape, relu, with_res)
    assert _fusable(x, m, res)
    xx = x.clone().requires_grad_(True)
    rr = res.clone().requires_grad_(True) if res is not None else None
    y = m(xx, rr)
    y.backward(dy)
    torch.cuda.synchronize()
    y0, dx0, dr0, dw0, db0, rm0, rv0 = _reference(m, x, res, dy, relu)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    # one bf16 rounding of the output
    torch.testing.assert_close(y.float(), y0, rtol=1e-2, atol=2e-2)
    torch.testing.assert_close(m.running_mean, rm0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m.running_var, rv0, rtol=1e-4, atol=1e-5)
    assert int(m.num_batches_tracked) == 1
    M = x.numel() // x.shape[1]
    # parameter grads are fp32 sums over M rows of bf16 data; the ReLU mask comes from the bf16
    # output, so an element whose fp32 pre-activation sits within bf16 rounding of 0 may differ
    scale = dy.float().abs().mean().item() * M ** 0.5
    torch.testing.assert_close(m.bias.grad, db0, rtol=2e-3, atol=2e-2 * scale)
    torch.testing.assert_close(m.weight.grad, dw0, rtol=2e-3, atol=2e-2 * scale)
    torch.testing.assert_close(xx.grad.float(), dx0, rtol=2e-2, atol=3e-2 * dx0.abs().max().item() + 1e-3)
    if res is not None:
        torch.testing.assert_close(rr.grad.float(), dr0, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("shape", [(4, 64, 9, 9), (3, 2048, 3, 3), (1, 8, 2, 3), (32, 128, 28, 28),
                                   (32, 64, 56, 56), (32, 2048, 7, 7), (31, 512, 14, 13)])
@pytest.mark.parametrize("relu,with_res", [(False, False), (True, False), (True, True), (False, True)])
def test_bnact_fp32_matches_fp32_reference(shape, relu, with_res):
    """fp32 activations (bench.py's default precision): two-kernel path, fp32 in and out."""
    assert _native.available()
    m, x, res, dy = _case(*shape, relu, with_res, dtype=torch.float32)
    assert _fusable(x, m, res)
    xx = x.clone().requires_grad_(True)
    rr = res.clone().requires_grad_(True) if res is not None else None
    y = m(xx, rr)
    y.backward(dy)
    torch.cuda.synchronize()
    y0, dx0, dr0, dw0, db0, rm0, rv0 = _reference(m, x, res, dy, relu)
    assert y.dtype == torch.float32 and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y, y0, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(m.running_mean, rm0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m.running_var, rv0, rtol=1e-4, atol=1e-5)
    M = x.numel() // x.shape[1]
    scale = dy.abs().mean().item() * M ** 0.5
    torch.testing.assert_close(m.bias.grad, db0, rtol=1e-4, atol=1e-4 * scale)
    torch.testing.assert_close(m.weight.grad, dw0, rtol=1e-4, atol=1e-4 * scale)
    torch.testing.assert_close(xx.grad, dx0, rtol=1e-3, atol=1e-4 * dx0.abs().max().item() + 1e-5)
    if res is not None:
        torch.testing.assert_close(rr.grad, dr0, rtol=1e-5, atol=1e-6)


@pytest.fixture
def single_launch():
    """The single-launch kernels are opt-in (GRACE_BN_FUSED=1); enable them for one test."""
    _native.lib().bn_set_fused(True)
    yield
    _native.lib().bn_set_fused(False)


def test_single_launch_path_selected(single_launch):
    """The co-resident single-launch kernels take the small/medium ResNet-50 shapes; the
    largest stage-1 shapes keep the two-kernel path."""
    C = _native.lib()
    for (n, c, h, w) in [(32, 128, 28, 28), (32, 2048, 7, 7), (32, 512, 14, 14)]:
        assert C.bn_fused_v(n * h * w, c, False) >= 8, (n, c, h, w)
        assert C.bn_fused_v(n * h * w, c, True) >= 8, (n, c, h, w)
    assert C.bn_fused_v(32 * 56 * 56, 64, False) == 16
    assert C.bn_fused_v(32 * 112 * 112, 64, False) == 0
    assert C.bn_fused_v(32 * 56 * 56, 256, True) == 0
    assert C.bn_fused_v(32 * 7 * 7, 512, False) == 0  # thin grid: two kernels are faster


@pytest.mark.parametrize("shape", [(32, 64, 56, 56), (32, 128, 28, 28), (32, 2048, 7, 7), (31, 512, 14, 13)])
@pytest.mark.parametrize("relu,with_res", [(False, False), (True, False), (True, True), (False, True)])
def test_bnact_single_launch_matches(shape, relu, with_res, single_launch):
    test_bnact_matches_fp32_reference(shape, relu, with_res)


def test_single_launch_matches_two_kernel_path():
    """Both layouts fold the same sums in a fixed (different) order: outputs agree to bf16
    rounding, statistics to fp32 rounding."""
    C = _native.lib()
    outs = []
    for fused in (True, False):
        C.bn_set_fused(fused)
        try:
            m, x, res, dy = _case(32, 128, 28, 28, True, True, seed=5)
            xx = x.clone().requires_grad_(True)
            y = m(xx, res)
            y.backward(dy)
            torch.cuda.synchronize()
            outs.append((y.float(), xx.grad.float(), m.weight.grad, m.bias.grad, m.running_var.clone()))
        finally:
            C.bn_set_fused(False)
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=1e-2, atol=2e-2)
    assert C.bn_spin_timeouts() == 0


def test_no_spin_timeouts():
    assert _native.lib().bn_spin_timeouts() == 0


@pytest.fixture
def deterministic():
    _native.lib().bn_set_deterministic(True)
    yield
    _native.lib().bn_set_deterministic(os.environ.get("GRACE_BN_DETERMINISTIC") == "1")


def test_bnact_graph_replay(deterministic):
    """Arrival counters re-arm in-kernel: repeated graph replays give the eager result bit for
    bit (fixed-order tree reductions; the default atomic backward is checked to tolerance below)."""
    m, x, res, dy = _case(8, 256, 14, 14, True, True, seed=3)
    xs = x.clone().requires_grad_(True)
    out = {}

    def step():
        xs.grad = None
        y = m(xs, res)
        y.backward(dy)
        return y

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            y_e = step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dx_e = xs.grad.clone()
    g = torch.cuda.CUDAGraph()
    # captured on the warm-up stream: xs's AccumulateGrad node (created in the warm-up backward)
    # runs on the stream it was created on -- no stream-mismatch sync inside the capture
    with torch.cuda.graph(g, stream=s):
        out["y"] = step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(out["y"], y_e, rtol=0, atol=0)
    torch.testing.assert_close(xs.grad, dx_e, rtol=0, atol=0)
    assert int(m.num_batches_tracked) == 2 + 3  # warmup + replays (the capture itself runs nothing)


def test_bnact_graph_replay_atomic(atomic_bn):
    """the atomic-totals backward under graph replay: the totals the forward zeroes are
    re-zeroed on every replay (replays match eager to fp32 summation order)"""
    m, x, res, dy = _case(8, 256, 14, 14, True, True, seed=3, dtype=torch.float32)
    xs = x.clone().requires_grad_(True)
    out = {}

    def step():
        xs.grad = None
        y = m(xs, res)
        y.backward(dy)
        return y

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dx_e = xs.grad.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out["y"] = step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(xs.grad, dx_e, rtol=1e-4, atol=1e-5 * float(dx_e.abs().max()))


def test_resnet_fused_step_as_accurate_as_unfused():
    """ResNet-18 forward/backward under bf16 autocast, fused BN path vs the unfused MIOpen path,
    both scored against an fp32 run of the same network.  (A random-init deep ResNet is chaotic:
    even two unfused bf16 runs differ through MIOpen's atomic reductions, and ResNet-50 at small
    batch decorrelates its first-layer gradients from rounding alone -- so the claim tested is
    "no less accurate than the stock path", not bitwise equality.)"""
    import os
    from grace_amd.models import resnet18

    torch.manual_seed(0)
    model = resnet18().to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 64, 64, device=DEV).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (8,), device=DEV)

    def run(force, amp):
        os.environ["GRACE_AMD_FORCE_TORCH"] = force
        try:
            model.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                loss = F.cross_entropy(model(x), y)
            loss.backward()
        finally:
            os.environ["GRACE_AMD_FORCE_TORCH"] = "0"
        return loss.detach().float(), torch.cat([p.grad.float().reshape(-1) for p in model.parameters()])

    l32, g32 = run("1", False)
    lf, gf = run("0", True)
    lu, gu = run("1", True)
    cf = F.cosine_similarity(gf, g32, dim=0).item()
    cu = F.cosine_similarity(gu, g32, dim=0).item()
    print(f"loss fp32 {l32.item():.5f} fused {lf.item():.5f} unfused {lu.item():.5f}; cos(fused, fp32) {cf:.4f} "
          f"cos(unfused, fp32) {cu:.4f}")
    assert abs(lf - l32) <= abs(lu - l32) + 2e-2
    assert cf >= cu - 0.03, (cf, cu)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8, 256, 14, 14), (4, 64, 28, 28)])
def test_bnact_dual_output_grads(dtype, shape):
    """dual=True: two aliases of the output, their gradients summed inside the fused backward
    kernels -- same dx / dres / dgamma / dbeta as one output whose gradient is dy1 + dy2."""
    m, x, res, dy = _case(*shape, relu=True, with_res=True, seed=3, dtype=dtype)
    g = torch.Generator(device="cpu").manual_seed(9)
    dy2 = torch.randn(shape, generator=g).to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    outs = []
    for dual in (False, True):
        xg = x.detach().clone().requires_grad_(True)
        rg = res.detach().clone().requires_grad_(True)
        m.zero_grad(set_to_none=True)
        y = m(xg, rg, dual=dual)
        if dual:
            y1, y2 = y
            assert y1.data_ptr() == y2.data_ptr()
            torch.autograd.backward([y1, y2], [dy, dy2])
        else:
            y.backward(dy + dy2)
        outs.append((xg.grad, rg.grad, m.weight.grad, m.bias.grad))
    tol = dict(rtol=1e-5, atol=1e-5) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    for i, (a, b) in enumerate(zip(*outs)):
        t = tol
        if dtype == torch.bfloat16 and i >= 2:
            # dgamma / dbeta sum M products: the unfused side rounds dy1 + dy2 to bf16 per element
            # first (the dual kernels add in fp32), a random-walk difference of ~sqrt(M) ulps
            t = dict(rtol=2e-2, atol=0.5)
        torch.testing.assert_close(a.float(), b.float(), **t)
    # only one alias used: its gradient alone
    xg = x.detach().clone().requires_grad_(True)
    y1, _ = m(xg, res, dual=True)
    y1.backward(dy)
    xr = x.detach().clone().requires_grad_(True)
    m(xr, res).backward(dy)
    torch.testing.assert_close(xg.grad.float(), xr.grad.float(), **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,k,s,p", [((4, 64, 56, 56), 3, 2, 1), ((2, 64, 15, 17), 3, 2, 1),
                                         ((2, 128, 8, 8), 2, 2, 0)])
def test_bn_relu_maxpool_fused_matches_reference(shape, k, s, p, dtype):
    """ResNet stem fusion (ops/bnact.py bn_relu_maxpool): pool(relu(bn(x))) forward and the
    gathered backward vs the fp32 PyTorch ops; running statistics updated as nn.BatchNorm2d."""
    from grace_amd.ops.bnact import bn_relu_maxpool
    from grace_amd.ops.pool import MaxPool2dNHWC

    m, x, _, _ = _case(*shape, relu=True, with_res=False, seed=4, dtype=dtype)
    pool = MaxPool2dNHWC(k, s, p)
    xa = x.detach().clone().requires_grad_(True)
    y = bn_relu_maxpool(xa, m, pool)
    xr = x.detach().float().requires_grad_(True)
    w = m.weight.detach().clone().requires_grad_(True)
    b = m.bias.detach().clone().requires_grad_(True)
    rm, rv = torch.zeros_like(m.running_mean), torch.ones_like(m.running_var)
    yr = F.max_pool2d(F.relu(F.batch_norm(xr, rm, rv, w, b, True, m.momentum, m.eps)), k, s, p)
    tol = dict(rtol=1e-4, atol=1e-4) if dtype == torch.float32 else dict(rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(y.float(), yr, **tol)
    torch.testing.assert_close(m.running_mean, rm, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(m.running_var, rv, rtol=1e-4, atol=1e-5)
    g = torch.Generator(device="cpu").manual_seed(8)
    dy = torch.randn(yr.shape, generator=g).to(DEV, dtype).contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    yr.backward(dy.float())
    if dtype == torch.float32:
        torch.testing.assert_close(xa.grad, xr.grad, rtol=1e-3, atol=1e-4)
        torch.testing.assert_close(m.weight.grad, w.grad, rtol=1e-3, atol=1e-3)
        torch.testing.assert_close(m.bias.grad, b.grad, rtol=1e-3, atol=1e-3)
    else:  # bf16 rounding may move an argmax: compare in aggregate
        rel = (xa.grad.float() - xr.grad).norm() / xr.grad.norm()
        assert rel < 0.05, rel
        torch.testing.assert_close(m.bias.grad, b.grad, rtol=5e-2, atol=0.5)


def test_bn_relu_maxpool_dual_output_sums_two_consumers_exactly():
    """dual=True: two aliases of the pooled output for two consumers (the first bottleneck's main
    path and shortcut); the max-pool backward sums their gradients itself -- bitwise the gradient of
    the single-output op fed with the autograd sum dy1 + dy2."""
    from grace_amd.ops.bnact import bn_relu_maxpool
    from grace_amd.ops.pool import MaxPool2dNHWC

    m, x, _, _ = _case(4, 64, 56, 56, relu=True, with_res=False, seed=5, dtype=torch.float32)
    pool = MaxPool2dNHWC(3, 2, 1)
    g = torch.Generator(device="cpu").manual_seed(9)
    shape = (4, 64, 28, 28)
    d1 = torch.randn(shape, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    d2 = torch.randn(shape, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    xa = x.detach().clone().requires_grad_(True)
    ya, yb = bn_relu_maxpool(xa, m, pool, dual=True)
    assert ya.data_ptr() == yb.data_ptr()
    torch.autograd.backward([ya, yb], [d1, d2])
    ga, wa = xa.grad.clone(), m.weight.grad.clone()
    m.weight.grad = None
    m.bias.grad = None
    xs = x.detach().clone().requires_grad_(True)
    y = bn_relu_maxpool(xs, m, pool)
    y.backward(d1 + d2)
    assert torch.equal(ga, xs.grad)
    torch.testing.assert_close(wa, m.weight.grad, rtol=0, atol=0)
    xo = x.detach().clone().requires_grad_(True)  # one consumer with a gradient, the other none
    y1, _ = bn_relu_maxpool(xo, m, pool, dual=True)
    y1.backward(d1)
    xp = x.detach().clone().requires_grad_(True)
    bn_relu_maxpool(xp, m, pool).backward(d1)
    assert torch.equal(xo.grad, xp.grad)


@pytest.fixture
def atomic_bn():
    prev = _native.lib().bn_atomic_chunks()
    _native.lib().bn_set_atomic_chunks(1 << 30)
    _native.lib().bn_set_deterministic(False)  # the suite default is the fixed-order tree
    yield
    _native.lib().bn_set_atomic_chunks(prev)
    _native.lib().bn_set_deterministic(os.environ.get("GRACE_BN_DETERMINISTIC") == "1")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,relu,with_res", [((32, 256, 14, 14), True, True), ((8, 2048, 7, 7), True, False),
                                                 ((16, 64, 28, 28), False, False)])
def test_bnact_atomic_and_tree_backward_agree(dtype, shape, relu, with_res, atomic_bn):
    """the opt-in atomic backward accumulates its two sums with fp32 atomics into totals the
    forward zeroed; a second backward through the same forward (retain_graph) must take the
    fixed-order tree instead -- both passes give the same gradients (so every grad doubles)"""
    m, x, res, dy = _case(*shape, relu, with_res, dtype=dtype)
    xx = x.clone().requires_grad_(True)
    rr = res.clone().requires_grad_(True) if res is not None else None
    y = m(xx, rr)
    y.backward(dy, retain_graph=True)
    g1 = [xx.grad.float().clone(), m.weight.grad.clone(), m.bias.grad.clone()]
    y.backward(dy)
    g2 = [xx.grad.float(), m.weight.grad, m.bias.grad]
    for a, b in zip(g1, g2):
        tol = 1e-4 * float(a.abs().max()) + 1e-6
        torch.testing.assert_close(b, 2 * a, rtol=1e-3 if dtype == torch.float32 else 2e-2,
                                   atol=tol if dtype == torch.float32 else 100 * tol)


def _run_bn(m, x, res, dy, dual, dy2):
    xx = x.clone().requires_grad_(True)
    rr = res.clone().requires_grad_(True) if res is not None else None
    out = m(xx, rr, dual=dual)
    if dual:
        torch.autograd.backward([out[0], out[1]], [dy, dy2])
        y = out[0]
    else:
        out.backward(dy)
        y = out
    torch.cuda.synchronize()
    return [y.detach().clone(), xx.grad.clone(), m.weight.grad.clone(), m.bias.grad.clone(),
            m.running_mean.clone(), m.running_var.clone()] + ([rr.grad.clone()] if rr is not None else [])


@pytest.mark.parametrize("shape", [(32, 128, 28, 28), (32, 256, 14, 14), (32, 512, 7, 7), (32, 2048, 7, 7),
                                   (32, 512, 14, 14), (32, 1024, 14, 14), (7, 256, 9, 11)])
@pytest.mark.parametrize("relu,with_res,dual", [(True, False, False), (True, True, True), (False, False, False),
                                                (False, True, False), (True, False, True)])
def test_bnact_fp32_single_launch_matches_two_kernel(shape, relu, with_res, dual):
    """fp32 single-launch kernels (rows held in registers, one co-resident launch per direction;
    opt-in: measured slower than the two-kernel path) give the two-kernel path's results up to
    the summation order of their differently chunked fixed-order trees."""
    C = _native.lib()
    n, c, h, w = shape
    m, x, res, dy = _case(*shape, relu, with_res, dtype=torch.float32)
    dy2 = torch.randn_like(dy) if dual else None
    got = None
    try:
        C.bn_set_fused_f32(True)
        vf, vb = C.bn_fused_v_f32(n * h * w, c, False), C.bn_fused_v_f32(n * h * w, c, True)
        got = []
        for _ in range(2):  # second call: the tile counters / generation words were re-armed
            m.weight.grad = m.bias.grad = None
            m.running_mean.zero_()
            m.running_var.fill_(1.0)
            got = _run_bn(m, x, res, dy, dual, dy2)
        C.bn_set_fused_f32(False)
        m.weight.grad = m.bias.grad = None
        m.running_mean.zero_()
        m.running_var.fill_(1.0)
        ref = _run_bn(m, x, res, dy, dual, dy2)
    finally:
        C.bn_set_fused_f32(False)
    if shape[0] == 32 and shape[1] != 1024:
        assert vf > 0 and vb > 0, (shape, vf, vb)  # the small ResNet-50 shapes take the fused path
    for a, b in zip(got, ref):
        tol = 1e-5 * float(b.abs().max()) + 1e-6
        assert float((a - b).abs().max()) <= tol
    assert C.bn_spin_timeouts() == 0
