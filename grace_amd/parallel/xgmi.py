"""``XgmiComm``: one-shot all-gather over xGMI peer memory for small compressed payloads.

The Allgather communicator's payloads are small (ResNet-50 Top-K 1 %: ~2 MB per rank).  A ring
all-gather moves each through W-1 sequential hops; on an 8 x MI355X node every GPU has a direct
xGMI link to every peer, so ``XgmiComm`` has every rank PULL each peer's payload over that
peer's own link, all links at once (SURVEY.md §5 "direct one-shot allgather";
csrc/comm/xgmi_allgather.hip has the protocol).  The reference gathers through Horovod/MPI
(/root/reference/grace_dl/dist/communicator/allgather.py:15-38).

    inner = RcclComm.from_process_group(inline=True)      # or TorchComm()
    comm = XgmiComm(inner, capacity_mb=8)                 # collective: every rank constructs it
    set_default_comm(comm)

* all-gathers whose per-rank payload fits the capacity (and is 16-B granular) run the native
  launches on the CURRENT stream (graph-capturable, no host sync); everything else (all-reduce,
  broadcast, all-to-all, larger gathers) goes to ``inner``.  The choice depends only on the byte
  size, identical on every rank (a misaligned or strided input is staged into an aligned
  scratch buffer instead of changing path on one rank);
* ``ranges`` (from the Allgather communicator, for capacity payloads with an in-band count):
  each peer's variable-length parts are pulled only up to the count the PEER wrote in its
  header -- the bytes on the links follow the real selection, not the capacity;
* ``payload_buffer``: ONE bucket's payload can be assembled straight in the exported slot
  (uncached regions), so that gather needs no staging copy;
* construction exchanges HIP IPC handles through the torch.distributed Store and, by default,
  verifies gathers against ``inner`` (every rank must agree, else it raises and the caller
  keeps ``inner``);
* a peer wait that exceeds the spin limit zero-fills that peer's rows, raises the process-wide
  fault flag (FusedSGD skips the update; parallel/health.py) and ``check()`` raises -- the
  device never hangs and no stale bytes reach the weights.
"""
from __future__ import annotations

import itertools

import torch
import torch.distributed as dist

from . import comm as _comm
from . import health as _health
from ..ops import _native

_UID = itertools.count()
_EMPTY_RANGES = torch.empty(0, 8, dtype=torch.int64)


def byte_ranges(specs, var, total: int = None) -> torch.Tensor:
    """The [k, 8] range table of a packed payload (``specs``: parallel.comm.Spec per tensor, in
    offset order) for XgmiPeers.all_gather.  ``var[i]`` = None (tensor i fixed) or
    ``(count_tensor, [esz0..esz3])``: tensor i's valid bytes are sum_j esz_j * hdr_j over the
    first four int32 words of tensor ``count_tensor``.  Gaps (alignment padding) are fixed; the
    last range runs to ``total`` (the packed buffer size)."""
    rows, end = [], 0
    for i, sp in enumerate(specs):
        start = sp.offset
        nxt = specs[i + 1].offset if i + 1 < len(specs) else None
        if start > end:
            rows.append([end, start - end, -1, 0, 0, 0, 0, 0])
            end = start
        stop = nxt if nxt is not None else (total if total is not None else -(-(start + sp.nbytes) // 16) * 16)
        v = var[i] if i < len(var) else None
        if v is None:
            rows.append([start, stop - start, -1, 0, 0, 0, 0, 0])
        else:
            ct, esz = v
            e = list(esz) + [0] * (4 - len(esz))
            rows.append([start, stop - start, specs[ct].offset] + e[:4] + [0])
        end = stop
    return torch.tensor(rows, dtype=torch.int64) if rows else _EMPTY_RANGES


class XgmiComm(_comm.Comm):
    _c = None  # not an RcclComm: GroupedComm issues the deferred gathers through all_gather_into
    accepts_ranges = True

    def __init__(self, inner: _comm.Comm, capacity_mb: float = 8.0, verify: bool = True, store=None,
                 spin_limit: int = 1 << 25, direct: bool = True):
        if not dist.is_initialized():
            raise RuntimeError("XgmiComm needs torch.distributed (its Store carries the IPC handles)")
        self.inner = inner
        self.rank, self.world_size = inner.rank, inner.world_size
        self.device = torch.cuda.current_device()
        _health.init()
        self._x = _native.lib().XgmiPeers(self.rank, self.world_size, self.device, int(capacity_mb * 2 ** 20),
                                          int(spin_limit))
        self._direct_ok = bool(direct)
        self._slot_owner = None
        self.direct_calls = 0
        if self._direct_ok and self._x.uncached:
            _comm.set_payload_provider(self.payload_buffer)
        store = store if store is not None else dist.distributed_c10d._get_default_store()
        key = f"grace_amd/xgmi/{next(_UID)}"
        store.set(f"{key}/{self.rank}", self._x.handle())
        handles = [bytes(store.get(f"{key}/{q}")) for q in range(self.world_size)]
        err = None
        try:
            self._x.open(handles)
        except RuntimeError as e:  # every rank must learn it: the peers would wait on this one
            err = e
        self._agree(err is None, f"xGMI peer mapping failed: {err}")
        self.capacity = int(self._x.capacity)
        self.one_shot_calls = 0
        if verify:
            self._verify()

    def __getattr__(self, name):  # stream, _mark, abort, ... of the wrapped comm
        inner = self.__dict__.get("inner")
        if inner is None:
            raise AttributeError(name)
        return getattr(inner, name)

    def _fits(self, inp: torch.Tensor) -> bool:
        # byte size and device only: the same answer on every rank
        n = inp.numel() * inp.element_size()
        return inp.is_cuda and n % 16 == 0 and 0 < n <= self.capacity

    @staticmethod
    def _aligned(t: torch.Tensor) -> bool:
        return t.is_contiguous() and t.data_ptr() % 16 == 0

    def payload_buffer(self, nbytes: int, key: str):
        """A uint8 [nbytes] view of the exported slot for ONE payload owner ``key`` (the same
        bucket every step), or None (not uncached, too large, or the slot is taken).  A payload
        assembled there is gathered without the staging copy."""
        if not (self._direct_ok and self._x.uncached) or nbytes <= 0 or nbytes > self.capacity or nbytes % 16:
            return None
        if self._slot_owner is None:
            self._slot_owner = key
        if self._slot_owner != key:
            return None
        return self._x.slot_tensor(int(nbytes))

    def all_gather_into(self, out, inp, async_op=False, ranges=None):
        if not self._fits(inp):
            return self.inner.all_gather_into(out, inp, async_op)
        o, i = out, inp
        if not self._aligned(i):  # staged, not a different path: every rank stays on the one-shot
            i = torch.empty(inp.numel() * inp.element_size(), dtype=torch.uint8, device=inp.device)
            i.copy_(inp.reshape(-1).view(torch.uint8))
        if not self._aligned(o):
            o = torch.empty(out.numel() * out.element_size(), dtype=torch.uint8, device=out.device)
        rg = ranges if ranges is not None else _EMPTY_RANGES
        # stream-ordered on the current stream: complete for every later op on it
        self._x.all_gather(o.reshape(-1).view(torch.uint8), i.reshape(-1).view(torch.uint8), rg)
        if o is not out:
            out.reshape(-1).view(torch.uint8).copy_(o)
        self.one_shot_calls += 1
        if i.data_ptr() == self._x.slot_ptr():
            self.direct_calls += 1
        return _comm.Work()

    def all_reduce(self, t, op="sum", async_op=False):
        return self.inner.all_reduce(t, op, async_op)

    def broadcast(self, t, src, async_op=False):
        return self.inner.broadcast(t, src, async_op)

    def all_to_all(self, out, inp, async_op=False):
        return self.inner.all_to_all(out, inp, async_op)

    def reduce_scatter(self, out, inp, op="sum", async_op=False):
        return self.inner.reduce_scatter(out, inp, op, async_op)

    def barrier(self):
        self.inner.barrier()

    def check(self):
        """Raise if a peer wait timed out (reads host-mapped words: no device sync, safe while
        capturing) or the inner comm reports an error."""
        _health.check()
        chk = getattr(self.inner, "check", None)
        if chk is not None:
            chk()

    def _verify(self):
        """Gather a rank-dependent pattern through both paths (two calls: both slots) and
        agree on the outcome across ranks; raise when any rank saw a mismatch."""
        dev = torch.device("cuda", self.device)
        ok = 1
        for salt in (1, 2):
            n = 4099 * 4  # odd count of 16-B vectors (exercises the grid-stride tails)
            inp = (torch.arange(n, device=dev, dtype=torch.int32) * (self.rank + 7) + salt * 1000003)
            got = torch.empty(self.world_size * n, dtype=torch.int32, device=dev)
            ref = torch.empty_like(got)
            self.all_gather_into(got, inp)
            self.inner.all_gather_into(ref, inp).wait()
            torch.cuda.synchronize(dev)
            ok &= int(torch.equal(got, ref)) & int(_health.status()[1] == 0)
        self._agree(bool(ok), "xGMI one-shot all-gather failed its self-check against the inner comm")
        self.one_shot_calls = 0

    def _agree(self, ok: bool, msg: str):
        """All ranks raise together (MIN over ranks through the inner comm) or none does."""
        dev = torch.device("cuda", self.device)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        self.inner.all_reduce(flag, "min").wait()
        torch.cuda.synchronize(dev)
        if int(flag.item()) != 1:
            raise RuntimeError(msg if not ok else "xGMI setup failed on a peer rank")

    def close(self):
        if _comm.get_payload_provider() == self.payload_buffer:
            _comm.set_payload_provider(None)
        self._x.close()
