"""Bounded payload capacity of the variable-size codecs (ops/cappayload.py).

The reference sends exactly the selected entries, padded to the largest rank's count after a
size all-gather (/root/reference/grace_dl/dist/communicator/allgather.py:15-38).  Here the
payload has a fixed capacity with an in-band count; with error feedback the auto capacity is a
small fraction of the tensor, entries past it SPILL into the residual and go out in later steps,
and the capacity grows (the same way on every rank) when steps overflow.
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(__file__))
from dist_utils import run_distributed  # noqa: E402


def test_threshold_spill_reappears_from_residual():
    """200 entries above the threshold, capacity 10 per step, zero gradients afterwards: every
    spilled entry is sent by a later step -- the sum of everything sent equals the input."""
    from grace_amd import grace_from_params
    from grace_amd.parallel.comm import LocalComm

    torch.manual_seed(0)
    n = 1000
    x0 = torch.zeros(n)
    big = torch.randperm(n)[:200]
    x0[big] = torch.randn(200).sign() * (0.5 + torch.rand(200))
    grc = grace_from_params({"compressor": "threshold", "threshold": 0.1, "capacity": 0.01, "memory": "residual",
                             "communicator": "allgather"}, comm=LocalComm())
    total = torch.zeros(n)
    sent_per_step = []
    for s in range(25):
        out = grc.step(x0.clone() if s == 0 else torch.zeros(n), "w")
        sent_per_step.append(int((out != 0).sum()))
        total += out
    assert max(sent_per_step) <= 10  # capacity ceil(0.01 * 1000)
    assert sent_per_step[0] == 10 and sum(sent_per_step) == 200
    torch.testing.assert_close(total, x0)
    assert float(grc.memory.residuals["w"].abs().max()) == 0.0


def test_threshold_auto_capacity_wire_bytes():
    """Default (auto) capacity with error feedback: <= 10 % of the uncompressed fp32 bytes."""
    from grace_amd import grace_from_params
    from grace_amd.parallel.comm import LocalComm

    n = 1 << 16
    grc = grace_from_params({"compressor": "threshold", "memory": "residual", "communicator": "allgather"},
                            comm=LocalComm())
    payload, _ = grc.compress_step(torch.randn(n) * 0.01, "w")
    wire = sum(t.numel() * t.element_size() for t in payload)
    assert wire <= 0.10 * 4 * n, wire
    # without error feedback the reference semantics stay exact (capacity 1.0, nothing spills)
    grc2 = grace_from_params({"compressor": "threshold", "communicator": "allgather"}, comm=LocalComm())
    x = torch.randn(n)
    torch.testing.assert_close(grc2.step(x.clone(), "v"), torch.where(x.abs() > 0.01, x, torch.zeros_like(x)))


def _grow_body(rank, world):
    from grace_amd import grace_from_params

    n = 4096
    grc = grace_from_params({"compressor": "threshold", "threshold": 0.5, "memory": "residual",
                             "communicator": "allgather", "world_size": world})
    comp = grc.compressor
    caps = []
    for s in range(4):
        g = torch.Generator().manual_seed(7 * s + rank)
        # rank 1 selects ~60 % of its entries, rank 0 almost none: only rank 1 overflows
        x = torch.randn(n, generator=g) * (2.0 if rank == 1 else 0.01)
        out = grc.step(x, "w")
        caps.append(comp.adaptive.cap["w"])
        t = out.contiguous()
        allv = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        assert all(torch.equal(a, allv[0]) for a in allv)  # identical result on every rank
    c = torch.tensor(caps, dtype=torch.int64)
    allc = [torch.empty_like(c) for _ in range(world)]
    dist.all_gather(allc, c)
    assert all(torch.equal(a, allc[0]) for a in allc), "ranks disagree on the capacity"
    assert caps[-1] > caps[0]  # grew after the overflowing step


def test_adaptive_capacity_grows_identically_on_every_rank_gloo():
    run_distributed(_grow_body, 2)


def test_inceptionn_auto_capacity_payload_size():
    from grace_amd import grace_from_params
    from grace_amd.parallel.comm import LocalComm

    n = 1 << 18  # buckets above 16K elements start at 1 byte per element
    # opt-in: the default is the lossless capacity 1.0 (INCEPTIONN has no error feedback)
    grc = grace_from_params({"compressor": "inceptionn", "communicator": "allgather", "capacity": "auto"},
                            comm=LocalComm())
    payload, _ = grc.compress_step(torch.randn(n) * 0.01, "w")
    wire = sum(t.numel() * t.element_size() for t in payload)
    assert wire <= 1.3 * n, wire  # was >= 4.25 n with capacity 1.0
    # exact against capacity 1.0 when the step fits
    x = torch.randn(n) * 0.01
    a = grace_from_params({"compressor": "inceptionn", "communicator": "allgather", "capacity": "auto"},
                          comm=LocalComm()).step(x, "q")
    b = grace_from_params({"compressor": "inceptionn", "communicator": "allgather", "capacity": 1.0},
                          comm=LocalComm()).step(x, "q")
    assert torch.equal(a, b)
    # the default payload is the lossless one
    d, _ = grace_from_params({"compressor": "inceptionn", "communicator": "allgather"},
                             comm=LocalComm()).compress_step(torch.randn(n) * 0.01, "w")
    assert sum(t.numel() * t.element_size() for t in d) >= 4 * n


def test_decode_ranks_cpu_path_rank_order_and_counts():
    """ops/cappayload.py decode_ranks on the CPU path: the output is zeroed, payloads are added in
    rank order (the sum order every rank reproduces), in-band counts bound each payload."""
    from grace_amd.ops import cappayload as P

    g = torch.Generator().manual_seed(4)
    n = 1000
    vals = [torch.randn(50, generator=g) for _ in range(3)]
    idxs = [torch.randperm(120, generator=g)[:50].to(torch.int32) for _ in range(3)]  # overlapping
    cnts = [None, torch.tensor([20, 50, 0, 0], dtype=torch.int32), torch.tensor([70, 50, 0, 0], dtype=torch.int32)]
    out = torch.full((n,), 9.0)
    P.decode_ranks(vals, idxs, cnts, out, 0.5)
    ref = torch.zeros(n)
    for v, i, k in zip(vals, idxs, (50, 20, 50)):  # rank 2's count 70 > capacity 50: the first 50
        for j in range(k):
            ref[int(i[j])] = ref[int(i[j])] + v[j] * 0.5
    assert torch.equal(out, ref)
