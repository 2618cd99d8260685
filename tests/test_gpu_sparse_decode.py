"""GPU numerics: the rank-ordered sparse decode (``cappayload.decode_ranks``: a zero fill plus one
native scatter launch per rank) against the plain fp32 PyTorch loop
``out = 0; out.index_add_(0, idx_r, v_r * s)`` for r = 0..W-1 -- including overlapping indices
across ranks, in-band counts (capacity payloads, overflow counted for the own payload only),
unaligned outputs and HIP-graph replay; and a W = 4 exchange (4 ranks on one GPU over gloo) whose
Top-K / Threshold decodes leave identical weights on every rank.

(The round-4 one-launch grid-barrier decode was deleted in round 5: it never beat this path inside
the whole-step graph, profiles/r4_final_headline_graph_kernels.txt.)"""
import os
import sys

import pytest
import torch

from grace_amd.ops import cappayload as P

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402

pytestmark = pytest.mark.gpu


def _payloads(W, n, k, seed, counts=False):
    g = torch.Generator().manual_seed(seed)
    vals, idxs, cnts = [], [], []
    for r in range(W):
        # every rank draws from the same first 2k positions: heavy cross-rank overlap
        pool = torch.randperm(min(n, 2 * k + 17), generator=g) if r % 2 == 0 else torch.randperm(n, generator=g)
        ix = pool[:k].to(torch.int32)
        vals.append(torch.randn(k, generator=g))
        idxs.append(ix)
        if counts:
            c = torch.zeros(4, dtype=torch.int32)
            c[0] = [k // 2, k, k + 5][r % 3]  # under, exactly at and over the capacity
            cnts.append(c)
        else:
            cnts.append(None)
    return vals, idxs, cnts


def _ref(vals, idxs, cnts, n, scale):
    out = torch.zeros(n)
    s = torch.tensor(scale, dtype=torch.float32)  # the kernel's fp32 scale (not a double multiply)
    for v, i, c in zip(vals, idxs, cnts):
        K = v.numel() if c is None else min(int(c[0]), v.numel())
        out.index_add_(0, i[:K].long(), v[:K] * s)
    return out


def _gpu(xs):
    return [None if x is None else x.cuda() for x in xs]


@pytest.mark.parametrize("W,n,k", [(1, 1000, 10), (3, 1_000_003, 20_000), (8, 257, 100), (20, 300_001, 3000)])
def test_decode_matches_fp32_reference(W, n, k):
    vals, idxs, cnts = _payloads(W, n, k, seed=W)
    out = torch.full((n,), 7.0, device="cuda")  # garbage: the decode zeroes
    P.decode_ranks(_gpu(vals), _gpu(idxs), cnts, out, 1.0 / W)
    torch.testing.assert_close(out.cpu(), _ref(vals, idxs, cnts, n, 1.0 / W), rtol=1e-6, atol=1e-7)
    again = torch.full((n,), -3.0, device="cuda")
    P.decode_ranks(_gpu(vals), _gpu(idxs), cnts, again, 1.0 / W)
    assert torch.equal(out, again)  # rank-ordered, atomic-free: the same bits on every call (and rank)


def test_decode_counts_unaligned_and_overflow():
    from grace_amd.parallel import health

    W, n, k = 5, 123_457, 4000
    vals, idxs, cnts = _payloads(W, n, k, seed=11, counts=True)
    health.init()
    over = [int(c[0]) > k for c in cnts]
    assert any(over) and not all(over)
    # counted exactly once per overflowing payload: only the decoding process's OWN payload
    # (every rank decodes every payload, so counting each would inflate W-fold)
    for own in [None] + list(range(W)):
        before = health.overflows()
        P.decode_ranks(_gpu(vals), _gpu(idxs), _gpu(cnts), torch.empty(n, device="cuda"), 0.5, own=own)
        torch.cuda.synchronize()
        assert health.overflows() == before + (0 if own is None else int(over[own])), own
    big = torch.full((n + 3,), -1.0, device="cuda")
    out = big[1:n + 1]  # 4-B aligned, not 16-B aligned
    P.decode_ranks(_gpu(vals), _gpu(idxs), _gpu(cnts), out, 0.5)
    torch.testing.assert_close(out.cpu(), _ref(vals, idxs, cnts, n, 0.5), rtol=1e-6, atol=1e-7)
    assert big[0].item() == -1.0 and big[n + 1].item() == -1.0 and big[n + 2].item() == -1.0


def test_decode_graph_replay():
    W, n, k = 4, 200_000, 5000
    vals, idxs, cnts = _payloads(W, n, k, seed=3)
    gv, gi = _gpu(vals), _gpu(idxs)
    out = torch.empty(n, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        P.decode_ranks(gv, gi, cnts, out, 0.25)
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        P.decode_ranks(gv, gi, cnts, out, 0.25)
    for step in range(3):
        vals2, idxs2, _ = _payloads(W, n, k, seed=50 + step)
        for a, b in zip(gv, vals2):
            a.copy_(b)
        for a, b in zip(gi, idxs2):
            a.copy_(b)
        graph.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(out.cpu(), _ref(vals2, idxs2, cnts, n, 0.25), rtol=1e-6, atol=1e-7)


def _w4_body(rank, world):
    from grace_amd import grace_from_params
    from grace_amd.parallel import DistributedOptimizer, FusedSGD
    from test_distributed_gloo import _same_on_all_ranks

    dev = torch.device("cuda", 0)
    for comp in ({"compressor": "topk", "compress_ratio": 0.05, "memory": "residual", "communicator": "allgather"},
                 {"compressor": "threshold", "threshold": 0.5, "memory": "residual", "communicator": "allgather"}):
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.ReLU(), torch.nn.Linear(256, 10)).to(dev)
        grc = grace_from_params(dict(comp, world_size=world))
        params = list(net.parameters())
        opt = DistributedOptimizer(FusedSGD(params, lr=0.1, momentum=0.5), grc,
                                   named_parameters=list(net.named_parameters()), bucket_cap_mb=0.05)
        g = torch.Generator().manual_seed(100 + rank)  # rank-specific data
        for _ in range(3):
            x = torch.randn(16, 64, generator=g).to(dev)
            opt.zero_grad()
            net(x).square().mean().backward()
            opt.step()
        torch.cuda.synchronize()
        for p in params:
            _same_on_all_ranks(p)
        opt.engine.remove()


def test_four_ranks_decode_identical():
    run_distributed(_w4_body, 4)
