"""Python face of the native RCCL runtime (csrc/comm/rccl_comm.cpp).

``RcclComm.from_process_group()`` bootstraps a dedicated RCCL communicator for GRACE traffic:
rank 0 creates the unique id, it travels through the torch.distributed Store (no extra
rendezvous), every rank calls ncclCommInitRank on its own GPU.  Collectives run on the
runtime's own high-priority HIP stream, ordered after the caller's current stream by an event;
``Work.wait()`` is stream-level (the host never blocks).  Select it for the default comm with
``GRACE_AMD_COMM=native``.

``inline=True`` (``GRACE_AMD_COMM=native-inline``) issues every collective on the caller's
CURRENT stream instead: no event fork/join, which is what a whole-step HIP graph with the
exchange on the main stream wants (bench.py picks it for ``--graph full`` without overlap; the
forked torch/ProcessGroupNCCL path measured 0.44 ms/step slower for ResNet-50 Top-K).

``RcclComm.tuned(nbytes)`` sizes the communicator's workgroup budget for the 7-link xGMI mesh
(one ring drives one outbound link per GPU, so a dense all-reduce needs several
channels): it builds one communicator per ``ncclConfig_t`` (minCTAs, maxCTAs) candidate, times an
all-reduce of the REAL bucket size on each, takes the MAX over ranks and keeps the fastest
(``choice`` records every candidate's time).
"""
from __future__ import annotations

import itertools
import weakref

import torch
import torch.distributed as dist

from . import comm as _comm
from ..ops import _native

_UID_COUNTER = itertools.count()
_EXIT_HOOKED = False
_LIVE = weakref.WeakSet()  # open RcclComm instances (graph.py picks thread-local capture while any is)


def live_count() -> int:
    """Open native RCCL communicators in this process."""
    return sum(1 for c in list(_LIVE) if c._c is not None)


def _hook_exit():
    global _EXIT_HOOKED
    if not _EXIT_HOOKED:
        import atexit

        atexit.register(_native.lib().rccl_mark_exiting)
        _EXIT_HOOKED = True


def _agree(ok: bool, group) -> None:
    """MIN of ``ok`` over the torch process group; every rank raises together on failure."""
    be = dist.get_backend(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if be == "nccl" else torch.device("cpu")
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if int(flag.item()) != 1:
        raise RuntimeError("native RCCL runtime failed its cross-rank self-check"
                           + ("" if not ok else " on a peer rank"))


class RcclComm(_comm.Comm):
    #: (minCTAs, maxCTAs) candidates of ``tuned``; (0, 0) = RCCL's own choice
    CTA_CANDIDATES = ((0, 0), (8, 8), (16, 16), (32, 32), (64, 64))

    def __init__(self, rank: int, world: int, unique_id: bytes, device: int, high_priority: bool = True,
                 inline: bool = False, ctas=(0, 0)):
        C = _native.lib()
        _hook_exit()
        self._c = C.RcclComm(rank, world, unique_id, device, high_priority, int(ctas[0]), int(ctas[1]))
        self.ctas = (int(ctas[0]), int(ctas[1]))
        self.choice = None
        self._c.inline = bool(inline)
        self.inline = bool(inline)
        self.rank, self.world_size, self.device = rank, world, device
        self._stream = torch.cuda.ExternalStream(self._c.stream_ptr, device=torch.device("cuda", device))
        _LIVE.add(self)

    @classmethod
    def tuned(cls, nbytes: int, group=None, candidates=None, iters: int = 10, inline: bool = False,
              high_priority: bool = True, dtype=torch.float32) -> "RcclComm":
        """The communicator whose (minCTAs, maxCTAs) budget all-reduces ``nbytes`` (the real dense
        bucket) fastest: every candidate is built (collectively), verified, timed on ``iters``
        all-reduces of that size (wall time around synchronised issue, MAX over ranks: the
        slowest rank sets each candidate's time), and all but the winner are destroyed.  Every
        rank takes the same decision.  ``choice`` = {"collective", "bytes", "ctas", "us": {cand: us}}."""
        import time

        cands = [tuple(c) for c in (candidates if candidates is not None else cls.CTA_CANDIDATES)]
        dev = torch.device("cuda", torch.cuda.current_device())
        n = max(1, int(nbytes) // torch.empty((), dtype=dtype).element_size())
        buf = torch.ones(n, dtype=dtype, device=dev)
        times, comms = {}, {}
        for cand in cands:
            c = cls.from_process_group(group, high_priority=high_priority, inline=False, ctas=cand)
            w = c._c.all_reduce(buf, "sum")  # warm: RCCL builds its channels / buffers lazily
            w.synchronize()
            c.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(iters):
                w = c._c.all_reduce(buf, "sum")
            w.synchronize()
            torch.cuda.synchronize(dev)
            t = torch.tensor([(time.perf_counter() - t0) * 1e6 / iters], dtype=torch.float64, device=dev)
            c._c.all_reduce(t, "max").synchronize()
            times[cand] = float(t.item())
            comms[cand] = c
        best = min(cands, key=lambda k: times[k])  # identical on every rank (MAX-reduced times)
        for cand, c in comms.items():
            if cand != best:
                c.close()
        win = comms[best]
        win._c.inline = bool(inline)
        win.inline = bool(inline)
        win.choice = {"collective": "all_reduce", "bytes": int(n * buf.element_size()),
                      "ctas": list(best), "us": {f"{a}/{b}": round(v, 2) for (a, b), v in times.items()}}
        return win

    @classmethod
    def from_process_group(cls, group=None, high_priority: bool = True, inline: bool = False,
                           verify: bool = True, timeout_s: float = 120.0, ctas=(0, 0)) -> "RcclComm":
        """Bootstrap the runtime from the torch.distributed Store; with ``verify`` (default) the
        new communicator passes :meth:`verify` on every rank before it is returned (all ranks
        raise together otherwise, so the caller can fall back to ``TorchComm``)."""
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed must be initialised (it provides the Store)")
        rank = dist.get_rank(group)
        world = dist.get_world_size(group)
        store = dist.distributed_c10d._get_default_store()
        key = f"grace_amd/rccl_uid/{next(_UID_COUNTER)}"
        if rank == 0:
            uid = _native.lib().rccl_unique_id()
            store.set(key, uid)
        else:
            uid = store.get(key)
        err = None
        c = None
        try:
            c = cls(rank, world, bytes(uid), torch.cuda.current_device(), high_priority, inline, ctas)
        except Exception as e:  # every rank must learn it (the peers would wait in verify)
            err = e
        if verify:
            ok = err is None and c.verify(timeout_s=timeout_s, agree=False)
            _agree(ok, group)
        elif err is not None:
            raise err
        if err is not None:
            raise err
        return c

    def _wait(self, w, deadline: float) -> None:
        import time

        while not w.is_completed():
            if time.monotonic() > deadline:
                self.abort(force=True)
                raise TimeoutError("native RCCL self-check: a collective did not complete")
            time.sleep(1e-3)

    def verify(self, timeout_s: float = 120.0, agree: bool = True) -> bool:
        """Cross-rank start-up self-check, run BEFORE any HIP-graph capture: an all-reduce, an
        all-gather and one grouped (all-gather + all-reduce) of rank-dependent data must produce
        the exact expected values on this rank, each within ``timeout_s`` (a host-side bounded
        wait: a collective that never completes aborts the communicator instead of hanging).
        With ``agree`` the verdict is MIN-reduced over the torch process group and every rank
        raises together on failure; returns this rank's verdict otherwise."""
        import time

        dev = torch.device("cuda", self.device)
        W, r = self.world_size, self.rank
        deadline = time.monotonic() + timeout_s
        ok = True
        try:
            a = torch.arange(4097, device=dev, dtype=torch.float32) + r
            self._wait(self._c.all_reduce(a, "sum"), deadline)
            ok &= torch.equal(a, torch.arange(4097, device=dev, dtype=torch.float32) * W + W * (W - 1) / 2)
            g_in = torch.full((1031,), r + 1, dtype=torch.int32, device=dev)
            g_out = torch.empty(1031 * W, dtype=torch.int32, device=dev)
            self._wait(self._c.all_gather(g_out, g_in), deadline)
            want = (torch.arange(W, device=dev, dtype=torch.int32) + 1).repeat_interleave(1031)
            ok &= torch.equal(g_out, want)
            b = torch.full((65,), float(r + 1), device=dev)
            g_out.zero_()
            self._wait(self._c.group([(g_out, g_in)], [b]), deadline)
            ok &= torch.equal(g_out, want) and torch.equal(b, torch.full_like(b, W * (W + 1) / 2))
            torch.cuda.synchronize(dev)
        except Exception:
            ok = False
        if agree:
            _agree(ok, None)
        return bool(ok)

    @property
    def nranks(self) -> int:
        """Ranks in the communicator as RCCL reports them (ncclCommCount)."""
        return int(self._c.nranks)

    @property
    def comm_device(self) -> int:
        """The device RCCL bound this rank's communicator to (ncclCommCuDevice)."""
        return int(self._c.comm_device)

    def set_inline(self, on: bool) -> None:
        """Issue on the caller's current stream (True) or the comm stream (False) from now on."""
        self._c.inline = bool(on)
        self.inline = bool(on)

    @property
    def stream(self) -> torch.cuda.Stream:
        return self._stream

    def _mark(self, *ts):
        if self.inline:  # same stream: the caching allocator's own ordering suffices
            return
        for t in ts:
            t.record_stream(self._stream)

    def _ret(self, w, async_op):
        if not async_op:
            w.wait()
            return _comm.Work()
        return _comm.Work([w])

    def all_reduce(self, t, op="sum", async_op=False):
        self._mark(t)
        return self._ret(self._c.all_reduce(t, op), async_op)

    def all_gather_into(self, out, inp, async_op=False):
        self._mark(out, inp)
        return self._ret(self._c.all_gather(out.view(-1), inp.view(-1)), async_op)

    def broadcast(self, t, src, async_op=False):
        self._mark(t)
        return self._ret(self._c.broadcast(t, src), async_op)

    def all_to_all(self, out, inp, async_op=False):
        self._mark(out, inp)
        return self._ret(self._c.all_to_all(out.view(-1), inp.view(-1)), async_op)

    def reduce_scatter(self, out, inp, op="sum", async_op=False):
        self._mark(out, inp)
        return self._ret(self._c.reduce_scatter(out, inp, op), async_op)

    def barrier(self):
        t = torch.zeros(1, device=torch.device("cuda", self.device))
        self._c.all_reduce(t, "sum").synchronize()

    def check(self):
        """Raise if RCCL reported an asynchronous error (peer failure, timeout)."""
        err = self._c.check_async_error()
        if err:
            raise RuntimeError(f"RCCL async error: {err}")

    def abort(self, force: bool = False) -> bool:
        """Abort the communicator (later issues fail).  Returns False when an issuing thread
        held it for > 5 s: that thread aborts on return (``force`` also aborts concurrently,
        see csrc/comm/rccl_comm.cpp)."""
        return bool(self._c.abort(force))

    def close(self):
        """Destroy the communicator now (before torch.distributed is torn down)."""
        self._c = None
