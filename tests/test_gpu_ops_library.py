"""GPU: the ``grace`` dispatcher operators run the native gfx950 kernels on cuda tensors and agree
with their CPU (PyTorch reference) registrations -- exactly for the deterministic codecs, in
distribution for the stochastic ones."""
import pytest
import torch

import grace_amd.ops  # noqa: F401
from grace_amd.ops import _native

pytestmark = pytest.mark.gpu
G = torch.ops.grace


def _g(n, seed=0):
    return torch.randn(n, generator=torch.Generator().manual_seed(seed))


def test_native_path_is_the_one_that_runs():
    assert _native.available() and _native.use_native(torch.empty(1, device="cuda"))


@pytest.mark.parametrize("n", [1000, 4099, 1 << 20])
def test_topk_compress_gpu_equals_cpu(n):
    g, r = _g(n), _g(n, 1) * 0.1
    vc, ic, rc = G.topk_compress(g, r, 0.01, 1.0, 1.0)
    vg, ig, rg = G.topk_compress(g.cuda(), r.cuda(), 0.01, 1.0, 1.0)
    oc, og = ic.long().argsort(), ig.long().cpu().argsort()
    assert torch.equal(ic.long()[oc], ig.long().cpu()[og])
    torch.testing.assert_close(vc[oc], vg.cpu()[og], rtol=0, atol=0)
    torch.testing.assert_close(rc, rg.cpu(), rtol=0, atol=0)
    dg = G.sparse_decompress(torch.stack([vg, vg]), torch.stack([ig, ig]), [n], 0.5)
    torch.testing.assert_close(dg.cpu(), G.sparse_decompress(vc, ic, [n], 1.0), rtol=0, atol=0)


def test_randomk_and_sign_gpu_equal_cpu():
    g = _g(100003)
    a = G.randomk_compress(g, 0.01, 99)
    b = G.randomk_compress(g.cuda(), 0.01, 99)
    torch.testing.assert_close(a, b.cpu(), rtol=0, atol=0)  # identical Feistel indices host / device
    rows = torch.stack([b, 2 * b])
    torch.testing.assert_close(G.randomk_decompress(rows, [100003], 0.01, 99, 0.5).cpu(),
                               G.randomk_decompress(rows.cpu(), [100003], 0.01, 99, 0.5), rtol=0, atol=0)
    w = G.sign_compress(g.cuda())
    assert torch.equal(w.cpu(), G.sign_compress(g))
    votes = torch.stack([w, w, G.sign_compress(-g.cuda())])
    assert torch.equal(G.sign_decompress(votes, [100003]).cpu(), torch.where(g >= 0, 1.0, -1.0))


def test_qsgd_and_natural_gpu_in_distribution():
    g = _g(4096).cuda()  # small n: |x| / ||x|| spans a few levels, so 128 roundings average well
    codes, norm = G.qsgd_compress(g, 127, 5)
    assert codes.dtype == torch.int8 and int(codes.abs().max()) <= 127
    torch.testing.assert_close(norm, torch.linalg.vector_norm(g).reshape(1))
    acc = torch.zeros_like(g)
    for s in range(128):
        c, n = G.qsgd_compress(g, 127, s)
        acc += G.qsgd_decompress(c, n, 127, [g.numel()])
    assert float((acc / 128 - g).abs().mean() / g.abs().mean()) < 0.05  # ~2 % expected
    x = g.abs() + 0.1
    dec = G.natural_decompress(G.natural_compress(x, 1), [x.numel()])
    lo = torch.exp2(torch.floor(torch.log2(x)))
    assert bool(torch.all((dec == lo) | (dec == 2 * lo)))
