"""Collective adapters (GRACE layer L1) for one-process-per-GPU data parallelism.

The reference talks to torch.distributed / Horovod directly from every communicator and even
from compressors (/root/reference/grace_dl/dist/communicator/*.py,
dist/compressor/powersgd.py:46-52, dist/memory/dgc.py:19).  Here all traffic goes through a
``Comm`` object that the Communicator owns and hands to the components that need it, so the
transport can be swapped:

* :class:`TorchComm`  - ``torch.distributed`` process group: RCCL over xGMI on MI355X
  (backend "nccl" *is* RCCL on ROCm), gloo on CPU for tests.
* :class:`LocalComm`  - world size 1 (collectives are identities, still no host sync).
* ``grace_amd.parallel.native_comm.RcclComm`` - the C++ RCCL runtime with its own
  communicator and dedicated comm stream (see csrc/comm/).

Payloads are *packed*: all tensors a compressor returns are moved as ONE flat byte buffer per
collective (zero-copy when the compressor already produced views of one allocation), instead
of one collective per payload tensor as in the reference.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

_ALIGN = 16


class Work:
    """Async handle: ``wait()`` blocks the *current stream* (not the host) on completion for
    GPU collectives, exactly like torch.distributed Work objects."""

    def __init__(self, works=None):
        self._works = [w for w in (works or []) if w is not None]

    def wait(self):
        for w in self._works:
            w.wait()
        self._works = []

    def is_completed(self) -> bool:
        return all(w.is_completed() for w in self._works)


class Comm:
    rank: int = 0
    world_size: int = 1

    def all_reduce(self, t: torch.Tensor, op: str = "sum", async_op: bool = False) -> Work:
        raise NotImplementedError

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False) -> Work:
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, src: int, async_op: bool = False) -> Work:
        raise NotImplementedError

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False) -> Work:
        """Chunk p of ``out`` <- chunk ``rank`` of rank p's ``inp`` (W equal chunks)."""
        raise NotImplementedError

    def barrier(self) -> None:
        pass


class LocalComm(Comm):
    """Single process: every collective is the identity."""

    def __init__(self):
        self.rank, self.world_size = 0, 1

    def all_reduce(self, t, op="sum", async_op=False):
        return Work()

    def all_gather_into(self, out, inp, async_op=False):
        out.view(-1)[: inp.numel()].copy_(inp.view(-1))
        return Work()

    def broadcast(self, t, src, async_op=False):
        return Work()

    def all_to_all(self, out, inp, async_op=False):
        out.view(-1).copy_(inp.view(-1))
        return Work()


_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}


class TorchComm(Comm):
    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self._gloo = self.backend == "gloo"

    def all_reduce(self, t, op="sum", async_op=False):
        w = dist.all_reduce(t, op=_OPS[op], group=self.group, async_op=async_op)
        return Work([w] if async_op else [])

    def all_gather_into(self, out, inp, async_op=False):
        if self._gloo:
            # gloo has no fused all_gather_into_tensor on all builds: use the list form
            chunks = list(out.view(self.world_size, -1).unbind(0))
            w = dist.all_gather(chunks, inp.view(-1), group=self.group, async_op=async_op)
        else:
            w = dist.all_gather_into_tensor(out.view(-1), inp.view(-1), group=self.group, async_op=async_op)
        return Work([w] if async_op else [])

    def broadcast(self, t, src, async_op=False):
        gsrc = dist.get_global_rank(self.group, src) if self.group is not None else src
        w = dist.broadcast(t, gsrc, group=self.group, async_op=async_op)
        return Work([w] if async_op else [])

    def all_to_all(self, out, inp, async_op=False):
        if self._gloo and out.is_cuda:  # gloo's all-to-all is host-only: stage through the CPU
            o = torch.empty(out.numel(), dtype=out.dtype)
            dist.all_to_all_single(o, inp.reshape(-1).cpu(), group=self.group)
            out.view(-1).copy_(o)
            return Work()
        w = dist.all_to_all_single(out.view(-1), inp.view(-1), group=self.group, async_op=async_op)
        return Work([w] if async_op else [])

    def barrier(self):
        dist.barrier(group=self.group)


class _LazyWork:
    """Work of a deferred collective: bound to the real handle when the group is flushed."""

    def __init__(self):
        self._w = None

    def bind(self, w):
        self._w = w

    def wait(self):
        if self._w is None:
            raise RuntimeError("collective still deferred: GroupedComm.flush() was not called")
        self._w.wait()

    def is_completed(self):
        return self._w is not None and self._w.is_completed()


class GroupedComm(Comm):
    """Defers the async sum all-reduces / all-gathers of a step and issues them together.

    Horovod's core negotiates and FUSES the tensors of many hooks into one transfer
    (/root/reference/patch_files/horovod/torch/mpi_ops.py:57-89, 407-439).  The bucketed engine
    already packs each bucket's payload into one buffer; with ``flush()`` the buckets' collectives
    of a whole step go out as ONE ``ncclGroupStart / ncclGroupEnd`` on the native RCCL runtime
    (csrc/comm/rccl_comm.cpp ``group``): RCCL schedules them concurrently over the xGMI links
    instead of one after the other.  Blocking collectives (PowerSGD's P/Q, DGC clipping) and
    broadcasts flush the pending group first, so the cross-rank order is unchanged.  On other
    comms the deferred ops are issued back to back at ``flush``.
    """

    def __init__(self, inner: Comm):
        self.inner = inner
        self.rank, self.world_size = inner.rank, inner.world_size
        self._pending = []

    def __getattr__(self, name):  # stream, check, abort, ... of the wrapped comm
        return getattr(self.inner, name)

    def all_reduce(self, t, op="sum", async_op=False):
        if not async_op or op != "sum" or not t.is_contiguous():
            self.flush()
            return self.inner.all_reduce(t, op, async_op)
        lw = _LazyWork()
        self._pending.append(("ar", t, None, lw, {}))
        return Work([lw])

    @property
    def accepts_ranges(self) -> bool:
        return bool(getattr(self.inner, "accepts_ranges", False))

    def all_gather_into(self, out, inp, async_op=False, ranges=None):
        kw = {"ranges": ranges} if ranges is not None else {}
        if not async_op:
            self.flush()
            return self.inner.all_gather_into(out, inp, async_op, **kw)
        lw = _LazyWork()
        self._pending.append(("ag", out, inp, lw, kw))
        return Work([lw])

    def broadcast(self, t, src, async_op=False):
        self.flush()
        return self.inner.broadcast(t, src, async_op)

    def all_to_all(self, out, inp, async_op=False):
        self.flush()
        return self.inner.all_to_all(out, inp, async_op)

    def barrier(self):
        self.flush()
        self.inner.barrier()

    @property
    def pending(self) -> int:
        return len(self._pending)

    def flush(self) -> None:
        if not self._pending:
            return
        pend, self._pending = self._pending, []
        native = getattr(self.inner, "_c", None)
        if native is not None and len(pend) > 1 and hasattr(native, "group"):
            gathers = [(o.view(-1), i.view(-1)) for k, o, i, _, _ in pend if k == "ag"]
            reduces = [t for k, t, _, _, _ in pend if k == "ar"]
            for k, a, b, _, _ in pend:
                self.inner._mark(*(x for x in (a, b) if x is not None))
            w = native.group(gathers, reduces)
            for _, _, _, lw, _ in pend:
                lw.bind(w)
            return
        for k, a, b, lw, kw in pend:
            w = self.inner.all_reduce(a, "sum", True) if k == "ar" else self.inner.all_gather_into(a, b, True, **kw)
            lw.bind(w)


def allgather_rows(comm: Comm, t: torch.Tensor, async_op: bool = False):
    """All-gather ``t`` along dim 0 when the first dimension differs per rank.

    Returns ``(work, finish)``; ``finish()`` (after ``work.wait()``) yields the rank-ordered
    concatenation.  The per-rank row counts travel in one tiny all-gather first (one host
    read: this is the path for data-dependent sizes -- sparse embedding gradients, Horovod's
    ``allgather`` -- never for the bucketed compressed exchange, which is fixed-size)."""
    W = comm.world_size
    if t.dim() == 0:
        t = t.view(1)
    t = t.contiguous()
    tail = tuple(t.shape[1:])
    row = 1
    for d in tail:
        row *= d
    cnt = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    cnts = torch.empty(W, dtype=torch.int64, device=t.device)
    comm.all_gather_into(cnts, cnt)
    sz = [int(v) for v in cnts.cpu().tolist()]
    mx = max(sz)
    send = torch.zeros(mx * row, dtype=t.dtype, device=t.device)
    send[: t.numel()].copy_(t.reshape(-1))
    out = torch.empty((W, mx * row), dtype=t.dtype, device=t.device)
    work = comm.all_gather_into(out, send, async_op=async_op)

    def finish():
        return torch.cat([out[r, : sz[r] * row].view((sz[r],) + tail) for r in range(W)], 0)

    return work, finish


_DEFAULT: Optional[Comm] = None


def default_comm() -> Comm:
    """The process-wide comm: torch.distributed WORLD if initialised, else LocalComm."""
    global _DEFAULT
    if _DEFAULT is not None:
        return _DEFAULT
    if dist.is_available() and dist.is_initialized():
        mode = os.environ.get("GRACE_AMD_COMM", "torch")
        if mode in ("native", "native-inline"):
            from .native_comm import RcclComm

            # one communicator per process (cached: every caller shares its stream)
            _DEFAULT = RcclComm.from_process_group(inline=mode == "native-inline")
            return _DEFAULT
        return TorchComm()
    return LocalComm()


def set_default_comm(comm: Optional[Comm]) -> None:
    global _DEFAULT
    _DEFAULT = comm


# ------------------------------------------------------------------------- payload packing
@dataclass(frozen=True)
class Spec:
    dtype: torch.dtype
    shape: Tuple[int, ...]
    offset: int  # bytes
    nbytes: int


def _align(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def make_specs(tensors: Sequence[torch.Tensor]) -> Tuple[List[Spec], int]:
    specs, off = [], 0
    for t in tensors:
        nb = _nbytes(t)
        specs.append(Spec(t.dtype, tuple(t.shape), off, nb))
        off = _align(off + nb)
    return specs, off


def _zero_copy_span(tensors: Sequence[torch.Tensor], specs: List[Spec], total: int) -> Optional[torch.Tensor]:
    """If the tensors already sit in one allocation with exactly the packed layout, return a
    uint8 view of that span (no copy)."""
    if not tensors:
        return None
    st = tensors[0].untyped_storage()
    base = tensors[0].data_ptr()
    for t, s in zip(tensors, specs):
        if not t.is_contiguous() or t.untyped_storage().data_ptr() != st.data_ptr():
            return None
        if t.data_ptr() - base != s.offset:
            return None
    start = base - st.data_ptr()
    if start + total > st.nbytes():
        total = specs[-1].offset + specs[-1].nbytes
        if start + total > st.nbytes():
            return None
    u8 = torch.empty(0, dtype=torch.uint8, device=tensors[0].device)
    u8.set_(st, start, (total,))
    return u8


def pack(tensors: Sequence[torch.Tensor]) -> Tuple[torch.Tensor, List[Spec]]:
    """Pack payload tensors into one uint8 buffer (16-B aligned sub-buffers)."""
    specs, total = make_specs(tensors)
    if total == 0:
        dev = tensors[0].device if tensors else "cpu"
        return torch.empty(0, dtype=torch.uint8, device=dev), specs
    z = _zero_copy_span(tensors, specs, total)
    if z is not None and z.numel() == total:
        return z, specs
    buf = torch.empty(total, dtype=torch.uint8, device=tensors[0].device)
    for t, s in zip(tensors, specs):
        if s.nbytes:
            buf[s.offset:s.offset + s.nbytes].copy_(t.contiguous().view(-1).view(torch.uint8))
    return buf, specs


def unpack(buf: torch.Tensor, specs: Sequence[Spec]) -> List[torch.Tensor]:
    out = []
    for s in specs:
        v = buf[s.offset:s.offset + s.nbytes]
        out.append(v.view(s.dtype).view(s.shape) if s.nbytes else torch.empty(s.shape, dtype=s.dtype, device=buf.device))
    return out


_PAYLOAD_PROVIDER = None


def set_payload_provider(fn) -> None:
    """``fn(nbytes, key) -> uint8 tensor or None``: where keyed payloads are assembled (the xGMI
    comm hands out its exported slot so that payload is gathered without a staging copy)."""
    global _PAYLOAD_PROVIDER
    _PAYLOAD_PROVIDER = fn


def get_payload_provider():
    return _PAYLOAD_PROVIDER


class PayloadBuilder:
    """Allocate a compressor's payload tensors as views of ONE buffer in the packed layout,
    so that ``pack`` is zero-copy and the whole payload moves in one collective.  With a ``key``
    (the bucket name) the registered payload provider may supply the buffer."""

    def __init__(self, device, entries: Sequence[Tuple[torch.dtype, Tuple[int, ...]]], key: Optional[str] = None):
        off, self._specs = 0, []
        for dt, shape in entries:
            n = 1
            for d in shape:
                n *= d
            nb = n * torch.empty((), dtype=dt).element_size()
            self._specs.append(Spec(dt, tuple(shape), off, nb))
            off = _align(off + nb)
        size = max(off, _ALIGN)
        buf = None
        if key is not None and _PAYLOAD_PROVIDER is not None and torch.device(device).type == "cuda":
            buf = _PAYLOAD_PROVIDER(size, key)
        self.buffer = buf if buf is not None else torch.empty(size, dtype=torch.uint8, device=device)
        self.tensors = unpack(self.buffer, self._specs)


def stack_rows(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """[W, n] view of W equally spaced same-shape 1-D views of one storage (zero-copy when the
    tensors are the per-rank slices of one all-gather output), else a stacked copy."""
    t0 = tensors[0].reshape(-1)
    if len(tensors) == 1:
        return t0.view(1, -1)
    n = t0.numel()
    st = t0.untyped_storage().data_ptr()
    es = t0.element_size()
    ok = all(t.is_contiguous() and t.numel() == n and t.dtype == t0.dtype and t.untyped_storage().data_ptr() == st
             for t in tensors)
    if ok:
        d = tensors[1].data_ptr() - tensors[0].data_ptr()
        if d > 0 and d % es == 0 and all(tensors[i + 1].data_ptr() - tensors[i].data_ptr() == d
                                          for i in range(len(tensors) - 1)):
            return torch.as_strided(t0, (len(tensors), n), (d // es, 1))
    return torch.stack([t.reshape(-1) for t in tensors])


def rank_rows(per_rank: Sequence[Sequence[torch.Tensor]]):
    """Describe W per-rank payloads as rank-strided rows of one byte buffer.

    Returns ``(base_u8, rank_stride_bytes, field_offsets_bytes)``: field f of rank r lives at
    byte ``r * rank_stride + field_offsets[f]`` of ``base_u8``.  Zero-copy when the payloads are
    the row views of one all-gather / broadcast output (the normal case); otherwise the
    payloads are packed into a fresh [W, span] buffer.
    """
    W = len(per_rank)
    first = [t for t in per_rank[0]]
    st0 = first[0].untyped_storage()
    starts = [p[0].data_ptr() for p in per_rank]
    offs = [t.data_ptr() - starts[0] for t in first]
    ok = all(len(p) == len(first) for p in per_rank)
    stride = starts[1] - starts[0] if W > 1 else 0
    if ok:
        for r, p in enumerate(per_rank):
            if starts[r] - starts[0] != r * stride:
                ok = False
                break
            for t, o in zip(p, offs):
                if t.untyped_storage().data_ptr() != st0.data_ptr() or t.data_ptr() - starts[r] != o:
                    ok = False
                    break
            if not ok:
                break
    if ok and (W == 1 or stride > 0):
        base = torch.empty(0, dtype=torch.uint8, device=first[0].device)
        start = starts[0] - st0.data_ptr()
        base.set_(st0, start, (st0.nbytes() - start,))
        return base, stride, offs
    bufs = [pack(list(p))[0] for p in per_rank]
    specs, span = make_specs(list(per_rank[0]))
    span = max(span, _ALIGN)
    out = torch.zeros(W * span, dtype=torch.uint8, device=first[0].device)
    for r, b in enumerate(bufs):
        out[r * span:r * span + b.numel()].copy_(b)
    return out, span, [s.offset for s in specs]
