"""The ``grace`` dispatcher operators (csrc/ops_library.cpp TORCH_LIBRARY(grace) + Meta kernels;
grace_amd/ops/library.py CPU / CUDA kernels): reference semantics on CPU, shape propagation
through meta / fake tensors, torch.library.opcheck, and tracing under torch.compile without a
graph break.  The GPU twin (native kernels vs these CPU results) is tests/test_gpu_ops_library.py."""
import pytest
import torch

import grace_amd.ops  # noqa: F401  (registers the kernels)
from grace_amd.ops import _native
from grace_amd.ops.library import k_of, ops

G = torch.ops.grace


def _g(n=4099, seed=0):
    return torch.randn(n, generator=torch.Generator().manual_seed(seed))


def test_every_op_is_registered_with_the_dispatcher():
    assert ops() == sorted(["topk_compress", "sparse_decompress", "randomk_compress", "randomk_decompress",
                            "sign_compress", "sign_decompress", "qsgd_compress", "qsgd_decompress",
                            "natural_compress", "natural_decompress"])
    for name in ops():
        op = getattr(G, name).default
        assert torch._C._dispatch_has_kernel_for_dispatch_key(op.name(), "CPU")
        assert torch._C._dispatch_has_kernel_for_dispatch_key(op.name(), "CUDA")
    if _native.available():  # the schemas come from the native library's TORCH_LIBRARY block
        assert torch._C._dispatch_has_kernel_for_dispatch_key("grace::topk_compress", "Meta")


def test_topk_compress_matches_reference_with_error_feedback():
    g, r = _g(), _g(seed=1) * 0.1
    vals, idx, res = G.topk_compress(g, r, 0.01, 0.5, 2.0)
    x = 0.5 * r + 2.0 * g  # ResidualMemory.compensate (reference residual.py:10-14)
    k = k_of(g.numel(), 0.01)
    assert vals.shape == (k,) and idx.dtype == torch.int32
    want = torch.topk(x.abs(), k).indices.sort().values
    assert torch.equal(idx.long().sort().values, want)
    torch.testing.assert_close(vals, x[idx.long()], rtol=0, atol=0)
    dec = G.sparse_decompress(vals, idx, list(g.shape), 1.0)
    torch.testing.assert_close(res + dec, x, rtol=0, atol=0)  # residual = x - decompress(compress(x))


def test_sparse_decompress_sums_ranks_in_order():
    v = torch.tensor([[1.0, 2.0], [10.0, 20.0]])
    i = torch.tensor([[0, 3], [3, 1]], dtype=torch.int32)
    out = G.sparse_decompress(v, i, [4], 0.5)
    torch.testing.assert_close(out, torch.tensor([0.5, 10.0, 0.0, 6.0]))


def test_randomk_same_indices_from_the_seed():
    g = _g()
    a = G.randomk_compress(g, 0.05, 42)
    b = G.randomk_compress(g * 2, 0.05, 42)
    torch.testing.assert_close(b, 2 * a)  # same positions on every "rank"
    dec = G.randomk_decompress(torch.stack([a, b]), list(g.shape), 0.05, 42, 1.0)
    nz = dec != 0
    assert int(nz.sum()) == k_of(g.numel(), 0.05)
    torch.testing.assert_close(dec[nz], 3 * g[nz])
    assert not torch.equal(G.randomk_compress(g, 0.05, 43), a)


def test_sign_majority_vote():
    g = _g(130)
    w = G.sign_compress(g)
    assert w.shape == (3,) and w.dtype == torch.int64
    torch.testing.assert_close(G.sign_decompress(w, [130]), torch.where(g >= 0, 1.0, -1.0))
    # two ranks vote +, one votes -: + wins (reference signsgd.py:25-30, ties go to +)
    rows = torch.stack([G.sign_compress(torch.ones(130)), G.sign_compress(torch.ones(130)),
                        G.sign_compress(-torch.ones(130))])
    assert torch.equal(G.sign_decompress(rows, [130]), torch.ones(130))


def test_qsgd_unbiased_and_typed():
    g = _g(2048)
    codes, norm = G.qsgd_compress(g, 127, 7)
    assert codes.dtype == torch.int8 and norm.shape == (1,)
    torch.testing.assert_close(norm, torch.linalg.vector_norm(g).reshape(1))
    assert G.qsgd_compress(g, 200, 7)[0].dtype == torch.int16
    # E[decompress(compress(x))] = x: average many independent roundings
    acc = torch.zeros_like(g)
    R = 64
    for s in range(R):
        c, n = G.qsgd_compress(g, 127, s)
        acc += G.qsgd_decompress(c, n, 127, [2048])
    err = (acc / R - g).abs().mean() / g.abs().mean()  # rounding noise / sqrt(R): ~2 %
    assert err < 0.05, err


def test_natural_powers_of_two_and_unbiased():
    g = _g(2048).abs() + 0.1
    codes = G.natural_compress(g, 3)
    dec = G.natural_decompress(codes, [2048])
    lo = torch.exp2(torch.floor(torch.log2(g)))
    assert torch.all((dec == lo) | (dec == 2 * lo))
    acc = sum(G.natural_decompress(G.natural_compress(g, s), [2048]) for s in range(64)) / 64
    assert ((acc - g).abs() / g).mean() < 0.05


def test_meta_and_fake_tensor_shapes():
    from torch._subclasses.fake_tensor import FakeTensorMode

    m = torch.empty(10000, device="meta")
    v, i, r = G.topk_compress(m, None, 0.01)
    assert v.shape == (100,) and i.dtype == torch.int32 and r.shape == m.shape and v.device.type == "meta"
    with FakeTensorMode():
        x = torch.empty(64, 65)
        assert G.sign_compress(x).shape == (65,)
        c, n = G.qsgd_compress(x, 200, 1)
        assert c.dtype == torch.int16 and c.shape == (4160,) and n.shape == (1,)
        assert G.natural_decompress(torch.empty(3, 4160, dtype=torch.uint8), [64, 65]).shape == (64, 65)
        assert G.randomk_decompress(torch.empty(2, 41), [64, 65], 0.01, 5, 1.0).shape == (64, 65)


@pytest.mark.parametrize("name,args", [
    ("topk_compress", lambda: (_g(1000), _g(1000, 1), 0.02, 1.0, 1.0)),
    ("sparse_decompress", lambda: (_g(8), torch.arange(8, dtype=torch.int32) * 3, [30], 0.5)),
    ("randomk_compress", lambda: (_g(1000), 0.05, 3)),
    ("sign_compress", lambda: (_g(1000),)),
    ("sign_decompress", lambda: (G.sign_compress(_g(1000)).repeat(3), [1000])),
    ("natural_decompress", lambda: (G.natural_compress(_g(100), 1).repeat(2), [100])),
])
def test_opcheck(name, args):
    """schema, fake (meta) kernel and device kernel agree (torch.library.opcheck)."""
    torch.library.opcheck(getattr(G, name).default, args(),
                          test_utils=("test_schema", "test_faketensor"))


def test_traces_under_torch_compile_without_graph_breaks():
    def step(g, r):
        v, i, r2 = G.topk_compress(g, r, 0.01, 1.0, 1.0)
        return G.sparse_decompress(v, i, [g.numel()], 1.0), r2

    fn = torch.compile(step, backend="aot_eager", fullgraph=True)
    g, r = _g(), torch.zeros(4099)
    out, r2 = fn(g, r)
    ref_out, ref_r2 = step(g, r)
    torch.testing.assert_close(out, ref_out)
    torch.testing.assert_close(r2, ref_r2)
