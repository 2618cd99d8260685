"""In-process simulation of W data-parallel ranks (survey 4, test plan item 4).

``LoopbackGroup(W)`` hands out W :class:`LoopbackComm` endpoints that implement the ``Comm``
interface with shared buffers and a barrier; ``run_ranks(fn, W)`` runs ``fn(rank, comm)`` on W
threads.  Communicator / compressor / engine logic can then be exercised for any W in one
process, on CPU or on one GPU, without process spawning or a rendezvous -- the CPU test suite
uses it next to the real multi-process gloo tests.

Collectives are synchronous (every endpoint blocks until all W arrived, results in rank order),
so ``async_op=True`` returns an already-completed ``Work``.
"""
from __future__ import annotations

import threading
from typing import Callable, List

import torch

from .comm import Comm, Work


class LoopbackGroup:
    def __init__(self, world_size: int, timeout: float = 60.0):
        self.world_size = world_size
        self.timeout = timeout
        self._barrier = threading.Barrier(world_size, timeout=timeout)
        self._slots: List[torch.Tensor] = [None] * world_size  # type: ignore[list-item]
        self._result = None

    def comm(self, rank: int) -> "LoopbackComm":
        return LoopbackComm(self, rank)

    def _exchange(self, rank: int, t: torch.Tensor) -> List[torch.Tensor]:
        """Every rank deposits ``t``; returns all ranks' tensors (rank order)."""
        self._slots[rank] = t.detach().clone()
        self._barrier.wait()
        out = list(self._slots)
        self._barrier.wait()  # nobody overwrites a slot before everyone has read it
        return out


_RED = {
    "sum": lambda ts: torch.stack(ts).sum(0),
    "max": lambda ts: torch.stack(ts).max(0).values,
    "min": lambda ts: torch.stack(ts).min(0).values,
}


class LoopbackComm(Comm):
    def __init__(self, group: LoopbackGroup, rank: int):
        self.group = group
        self.rank = rank
        self.world_size = group.world_size

    def all_reduce(self, t, op="sum", async_op=False):
        ts = self.group._exchange(self.rank, t)
        t.copy_(_RED[op]([x.to(t.device) for x in ts]).to(t.dtype))
        return Work()

    def all_gather_into(self, out, inp, async_op=False):
        ts = self.group._exchange(self.rank, inp.reshape(-1))
        out.view(self.world_size, -1).copy_(torch.stack([x.to(out.device) for x in ts]))
        return Work()

    def broadcast(self, t, src, async_op=False):
        ts = self.group._exchange(self.rank, t)
        t.copy_(ts[src].to(t.device))
        return Work()

    def reduce_scatter(self, out, inp, op="sum", async_op=False):
        ts = self.group._exchange(self.rank, inp.reshape(-1))
        red = _RED[op]([x.to(out.device) for x in ts]).view(self.world_size, -1)
        out.view(-1).copy_(red[self.rank])
        return Work()

    def all_to_all(self, out, inp, async_op=False):
        ts = self.group._exchange(self.rank, inp.reshape(-1))
        W = self.world_size
        out.view(W, -1).copy_(torch.stack([x.to(out.device).view(W, -1)[self.rank] for x in ts]))
        return Work()

    def barrier(self):
        self.group._barrier.wait()


def run_ranks(fn: Callable[[int, Comm], object], world_size: int, timeout: float = 120.0) -> list:
    """Run ``fn(rank, comm)`` on ``world_size`` threads; returns the per-rank results and
    re-raises the first failure."""
    group = LoopbackGroup(world_size, timeout=timeout)
    results = [None] * world_size
    errors: list = []

    def body(r):
        try:
            results[r] = fn(r, group.comm(r))
        except BaseException as e:  # noqa: BLE001 - re-raised in the caller
            errors.append((r, e))
            group._barrier.abort()

    threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(world_size)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout)
    if errors:
        r, e = sorted(errors, key=lambda x: isinstance(x[1], threading.BrokenBarrierError))[0]
        raise RuntimeError(f"rank {r} failed: {e!r}") from e
    return results
