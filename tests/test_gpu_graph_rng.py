"""Device step counters for stochastic codecs (graph-replay-safe randomness).

* a kernel fed (base seed, device step s) produces exactly what it produces for the host-mixed
  seed ``base ^ s * golden`` -- the SeedArg mixing is bit-identical to ops.randomk.mix_step;
* a HIP graph that captured a compress call draws NEW randomness on every replay (the captured
  ``add_(1)`` advances the counter) and stays self-consistent (Random-K decompress scatters to
  the indices the same replay gathered from);
* state_dict() folds replayed steps back into the host counters.
"""
import pytest
import torch

from grace_amd import compressor as Z
from grace_amd.core import register_layout
from grace_amd.ops import powersgd as PS
from grace_amd.ops import quant as Q
from grace_amd.ops import randomk as R
from grace_amd.ops.layout import SegmentLayout
from grace_amd.ops.randomk import mix_step

pytestmark = pytest.mark.gpu

SHAPES = [(33, 17), (4096,), (100003,), (5,)]
BASE = 0x1234_5678_9ABC_DEF1


def _bucket(name="rng_bucket", seed=0):
    g = torch.Generator().manual_seed(seed)
    ts = [torch.randn(*s, generator=g) for s in SHAPES]
    lay = SegmentLayout.from_tensors(ts)
    register_layout(name, lay)
    return torch.cat([t.flatten() for t in ts]).cuda(), lay


def _step(v):
    return torch.tensor([v], dtype=torch.int64, device="cuda")


def test_device_step_equals_host_mixed_seed():
    x, lay = _bucket()
    step = 7
    mixed = mix_step(BASE, step)
    norms = torch.stack([x[o:o + n].norm() for _, o, n in lay.segments()]).float().contiguous()
    a = torch.empty(lay.total, dtype=torch.int8, device="cuda")
    b = torch.empty_like(a)
    Q.qsgd_quantize(x, lay, norms, 64, BASE, a, step=_step(step))
    Q.qsgd_quantize(x, lay, norms, 64, mixed, b)
    assert torch.equal(a, b)
    c1 = torch.empty(lay.total, dtype=torch.uint8, device="cuda")
    c2 = torch.empty_like(c1)
    Q.natural_encode(x, BASE, c1, step=_step(step))
    Q.natural_encode(x, mixed, c2)
    assert torch.equal(c1, c2)
    torch.testing.assert_close(PS.randn_shared(4099, BASE, "cuda", step=_step(step)),
                               PS.randn_shared(4099, mixed, "cuda"), rtol=0, atol=0)
    ks = [max(1, n // 10) for _, _, n in lay.segments()]
    seeds = [BASE ^ i for i in range(lay.n_seg)]
    v1 = R.gather(x, lay, ks, seeds, step=step, step_t=_step(step))
    v2 = R.gather(x, lay, ks, seeds, step=step)
    v3 = R.gather(x.cpu(), lay, ks, seeds, step=step)  # torch Feistel: same indices
    assert torch.equal(v1, v2)
    assert torch.equal(v1.cpu(), v3)


def _capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = fn()
    torch.cuda.synchronize()
    return g, out


@pytest.mark.parametrize("make", [lambda: Z.QSGDCompressor(16), lambda: Z.TernGradCompressor(),
                                  lambda: Z.NaturalCompressor()])
def test_graph_replay_draws_fresh_rounding(make):
    x, _ = _bucket()
    comp = make()

    def fn():
        payload, ctx = comp.compress(x, "rng_bucket")
        return payload[0]

    g, out = _capture(fn)
    seen = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        seen.append(out.clone())
    assert not torch.equal(seen[0], seen[1]) and not torch.equal(seen[1], seen[2])
    # the counter counts EXECUTED compress calls: 2 warm-up + 3 replays (the capture-time call
    # only records the graph); state_dict() folds it back into the host dict
    comp.state_dict()
    assert comp.steps["rng_bucket"] == 5


def test_graph_replay_randomk_roundtrip_consistent():
    x, lay = _bucket()
    comp = Z.RandomKCompressor(0.05)

    def fn():
        payload, ctx = comp.compress(x, "rng_bucket")
        return comp.decompress(payload, ctx)

    g, out = _capture(fn)
    masks = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        nz = out != 0
        # decompress put exactly the gathered values back at the gathered indices
        assert torch.equal(out[nz], x[nz])
        masks.append(nz.clone())
    assert not torch.equal(masks[0], masks[1])
    assert int(masks[0].sum()) == int(masks[2].sum())


def test_graph_replay_powersgd_post_bump_counter():
    """PowerSGD advances its device step counter inside the P = M Q launch (no add_ kernel):
    every replay still draws a fresh Q (a new P) and state_dict() reports executed steps."""
    x, _ = _bucket()
    comp = Z.PowerSGDCompressor(rank=2)

    def fn():
        payload, ctx = comp.compress(x, "rng_bucket")
        return ctx.extra["p"]

    g, out = _capture(fn)
    seen = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        seen.append(out.clone())
    assert not torch.equal(seen[0], seen[1]) and not torch.equal(seen[1], seen[2])
    comp.state_dict()
    assert comp.steps["rng_bucket"] == 5
    # the next eager step continues the sequence: the same Q as a fresh compressor at step 6
    ref = Z.PowerSGDCompressor(rank=2)
    ref.steps["rng_bucket"] = 5
    torch.testing.assert_close(fn(), ref.compress(x, "rng_bucket")[1].extra["p"], rtol=0, atol=0)
