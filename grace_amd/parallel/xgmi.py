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
* a peer wait that exceeds the spin limit fills that peer's rows (zeros = an empty payload for a
  gather, NaN for the gather-reduce all-reduce), raises the process-wide fault flag (FusedSGD
  skips the update; parallel/health.py) and ``check()`` raises -- the device never hangs and no
  stale bytes reach the weights.
"""
from __future__ import annotations

import itertools

import torch
import torch.distributed as dist

from . import comm as _comm
from . import health as _health
from ..ops import _native

_UID = itertools.count()


def n_bytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()
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
                 spin_limit: int = 1 << 25, direct: bool = True, select: str = "size"):
        """``select``: "size" = every gather that fits the capacity takes the one-shot path;
        "probe" = the FIRST eager gather of each payload size times both paths (the one-shot pull
        and ``inner``'s all-gather, e.g. RCCL's ring) on that exact size, every rank takes the MAX
        over ranks of each and all pick the faster one (``choices`` records it) -- the path
        choice for the 7-link mesh is measured, not assumed."""
        if not dist.is_initialized():
            raise RuntimeError("XgmiComm needs torch.distributed (its Store carries the IPC handles)")
        self.inner = inner
        self.rank, self.world_size = inner.rank, inner.world_size
        self.device = torch.cuda.current_device()
        _health.init()
        self._x = _native.lib().XgmiPeers(self.rank, self.world_size, self.device, int(capacity_mb * 2 ** 20),
                                          int(spin_limit))
        if select not in ("size", "probe"):
            raise ValueError(f"select must be 'size' or 'probe', not {select!r}")
        self.select = select
        self.choices = {}  # payload bytes -> {"path": "xgmi" | "inner", "xgmi_us": .., "inner_us": ..}
        self._direct_ok = bool(direct)
        self._slot_owner = None
        self._owner_seen = 0   # payload_buffer calls when the owner last asked
        self._buf_calls = 0
        self.direct_calls = 0
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
        # direct slot writes only where EVERY rank got an uncached region (the kernel also reads
        # each peer's published slot choice, so a disagreement could not read stale bytes, but
        # uniform behaviour keeps the per-rank work and the bench labels identical)
        self._direct_ok = self._all(self._direct_ok and bool(self._x.uncached))
        if self._direct_ok:
            _comm.set_payload_provider(self.payload_buffer)
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
        self._buf_calls += 1
        # the owner is whoever asks first; an owner that stopped asking (e.g. a DDP bucket name
        # retired by re-bucketing, ddp_hook.py `.g{n}` generations) hands the slot on after
        # _OWNER_IDLE calls by other keys.  Every rank sees the same key sequence, and the pull
        # kernel reads each peer's published slot anyway (csrc/comm/xgmi_allgather.hip)
        if self._slot_owner is not None and self._slot_owner != key and \
                self._buf_calls - self._owner_seen > self._OWNER_IDLE:
            self._slot_owner = None
        if self._slot_owner is None:
            self._slot_owner = key
        if self._slot_owner != key:
            return None
        self._owner_seen = self._buf_calls
        return self._x.slot_tensor(int(nbytes))

    _OWNER_IDLE = 16

    def _choose(self, out, inp) -> str:
        """"xgmi" or "inner" for this payload size (identical on every rank: decided from
        MAX-reduced timings in an eager call, or by size alone)."""
        nbytes = inp.numel() * inp.element_size()
        if self.select != "probe":
            return "xgmi"
        c = self.choices.get(nbytes)
        if c is not None:
            return c["path"]
        if torch.cuda.is_current_stream_capturing():
            # a size first seen inside a capture (the eager warm-up normally saw it): every rank
            # is in the same capture, so the size rule is still rank-consistent
            return "xgmi"
        c = self.choices[nbytes] = self._probe(out, inp)
        return c["path"]

    def _probe(self, out, inp, iters: int = 8) -> dict:
        dev = torch.device("cuda", self.device)
        o = torch.empty_like(out)
        i = inp.detach().clone() if self._aligned(inp) else inp.contiguous().clone()
        import time

        times = []
        for path in ("xgmi", "inner"):
            fn = (lambda: self._one_shot(o, i, None)) if path == "xgmi" else \
                (lambda: self.inner.all_gather_into(o, i, False).wait())
            fn()  # warm (RCCL lazily builds its channels for a new size)
            torch.cuda.synchronize(dev)
            self.inner.barrier()
            torch.cuda.synchronize(dev)
            # wall time around synchronised issue: also right for a host-driven inner (gloo)
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize(dev)
            times.append((time.perf_counter() - t0) * 1e6 / iters)
        t = torch.tensor(times, dtype=torch.float64, device=dev)
        self.inner.all_reduce(t, "max").wait()  # the slowest rank sets each path's time
        torch.cuda.synchronize(dev)
        xg, inn = (float(v) for v in t.tolist())
        self.one_shot_calls -= iters + 1
        return {"path": "xgmi" if xg <= inn else "inner", "xgmi_us": round(xg, 2), "inner_us": round(inn, 2),
                "bytes": int(inp.numel() * inp.element_size()), "collective": "all_gather"}

    def all_gather_into(self, out, inp, async_op=False, ranges=None):
        if not self._fits(inp) or self._choose(out, inp) != "xgmi":
            return self.inner.all_gather_into(out, inp, async_op)
        return self._one_shot(out, inp, ranges)

    def _one_shot(self, out, inp, ranges, fill: int = 0):
        o, i = out, inp
        if not self._aligned(i):  # staged, not a different path: every rank stays on the one-shot
            i = torch.empty(inp.numel() * inp.element_size(), dtype=torch.uint8, device=inp.device)
            i.copy_(inp.reshape(-1).view(torch.uint8))
        if not self._aligned(o):
            o = torch.empty(out.numel() * out.element_size(), dtype=torch.uint8, device=out.device)
        rg = ranges if ranges is not None else _EMPTY_RANGES
        # stream-ordered on the current stream: complete for every later op on it
        self._x.all_gather(o.reshape(-1).view(torch.uint8), i.reshape(-1).view(torch.uint8), rg, fill)
        if o is not out:
            out.reshape(-1).view(torch.uint8).copy_(o)
        self.one_shot_calls += 1
        if i.data_ptr() == self._x.slot_ptr():
            self.direct_calls += 1
        return _comm.Work()

    def all_reduce(self, t, op="sum", async_op=False):
        """Small all-reduces as a one-shot gather + a rank-ordered local reduction (the same bytes
        summed in the same order on every rank: bit-identical results); larger ones -- or when
        ``select="probe"`` measured ``inner`` faster for this size -- go to ``inner``."""
        n = t.numel() * t.element_size()
        # sizes that are not 16-B granular (PowerSGD's P / Q: rows x rank fp32) are padded, not
        # sent to the inner comm: the path must not depend on the byte size's alignment (a gloo
        # inner cannot be captured, and every rank must take the same path)
        if (op not in ("sum", "max", "min") or not t.is_contiguous() or not t.is_floating_point()
                or not t.is_cuda or n == 0 or -(-n // 16) * 16 > self.capacity):
            return self.inner.all_reduce(t, op, async_op)
        if self.select == "probe":
            c = self.choices.get(("ar", n))
            if c is None:
                if torch.cuda.is_current_stream_capturing():
                    c = {"path": "xgmi"}
                else:
                    c = self.choices[("ar", n)] = self._probe_reduce(t, op)
            if c["path"] != "xgmi":
                return self.inner.all_reduce(t, op, async_op)
        self._gather_reduce(t, op)
        return _comm.Work()

    def _gather_reduce(self, t, op):
        n, esz = t.numel(), t.element_size()
        npad = -(-(n * esz) // 16) * 16 // esz  # 16-B granular row
        src = t.reshape(-1)
        if npad != n:
            src = torch.zeros(npad, dtype=t.dtype, device=t.device)
            src[:n].copy_(t.reshape(-1))
        rows = torch.empty((self.world_size, npad), dtype=t.dtype, device=t.device)
        # a timed-out peer's rows come back as NaN (not zeros): the reduced value is visibly
        # wrong for ANY consumer, not only for FusedSGD's fault-word check
        self._one_shot(rows.view(-1), src, None, fill=0xFFFFFFFF)
        if npad != n:
            rows = rows[:, :n]
        if op == "sum":
            torch.sum(rows, 0, out=t.view(-1))
        elif op == "max":
            torch.amax(rows, 0, out=t.view(-1))
        else:
            torch.amin(rows, 0, out=t.view(-1))

    def _probe_reduce(self, t, op, iters: int = 8) -> dict:
        import time

        dev = torch.device("cuda", self.device)
        buf = t.detach().clone()
        times = []
        for path in ("xgmi", "inner"):
            def fn():
                buf.copy_(t)
                if path == "xgmi":
                    self._gather_reduce(buf, op)
                else:
                    self.inner.all_reduce(buf, op, False).wait()
            fn()
            torch.cuda.synchronize(dev)
            self.inner.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize(dev)
            times.append((time.perf_counter() - t0) * 1e6 / iters)
        tt = torch.tensor(times, dtype=torch.float64, device=dev)
        self.inner.all_reduce(tt, "max").wait()
        torch.cuda.synchronize(dev)
        xg, inn = (float(v) for v in tt.tolist())
        self.one_shot_calls -= iters + 1
        return {"path": "xgmi" if xg <= inn else "inner", "xgmi_us": round(xg, 2), "inner_us": round(inn, 2),
                "bytes": int(t.numel() * t.element_size()), "collective": "all_reduce"}

    def broadcast(self, t, src, async_op=False):
        return self.inner.broadcast(t, src, async_op)

    def all_to_all(self, out, inp, async_op=False):
        """out[p] = chunk ``rank`` of rank p's ``inp`` (QSGD's compressed-domain reduce-scatter):
        each rank pulls only its own chunk of every peer's staged payload, all links at once
        (graph-capturable); sizes past the capacity / not 16-B x W granular -- or, with
        ``select="probe"``, sizes where ``inner`` measured faster -- go to ``inner``."""
        n = inp.numel() * inp.element_size()
        if not (inp.is_cuda and 0 < n <= self.capacity and n % (16 * self.world_size) == 0
                and out.numel() * out.element_size() == n):
            return self.inner.all_to_all(out, inp, async_op)
        if self.select == "probe":
            c = self.choices.get(("a2a", n))
            if c is None:
                if torch.cuda.is_current_stream_capturing():
                    c = {"path": "xgmi"}
                else:
                    c = self.choices[("a2a", n)] = self._probe_a2a(out, inp)
            if c["path"] != "xgmi":
                return self.inner.all_to_all(out, inp, async_op)
        self._a2a(out, inp)
        return _comm.Work()

    def _a2a(self, out, inp):
        i = inp if self._aligned(inp) else inp.contiguous().clone()
        o = out if self._aligned(out) else torch.empty(out.numel() * out.element_size(), dtype=torch.uint8,
                                                       device=out.device)
        self._x.all_to_all(o.reshape(-1).view(torch.uint8), i.reshape(-1).view(torch.uint8))
        if o is not out:
            out.reshape(-1).view(torch.uint8).copy_(o)
        self.one_shot_calls += 1

    def _probe_a2a(self, out, inp, iters: int = 8) -> dict:
        import time

        dev = torch.device("cuda", self.device)
        o = torch.empty_like(out)
        i = inp.detach().clone()
        times = []
        for path in ("xgmi", "inner"):
            fn = (lambda: self._a2a(o, i)) if path == "xgmi" else (lambda: self.inner.all_to_all(o, i, False).wait())
            fn()
            torch.cuda.synchronize(dev)
            self.inner.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(iters):
                fn()
            torch.cuda.synchronize(dev)
            times.append((time.perf_counter() - t0) * 1e6 / iters)
        tt = torch.tensor(times, dtype=torch.float64, device=dev)
        self.inner.all_reduce(tt, "max").wait()
        torch.cuda.synchronize(dev)
        xg, inn = (float(v) for v in tt.tolist())
        self.one_shot_calls -= iters + 1
        return {"path": "xgmi" if xg <= inn else "inner", "xgmi_us": round(xg, 2), "inner_us": round(inn, 2),
                "bytes": int(n_bytes(inp)), "collective": "all_to_all"}

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
        """Gather a rank-dependent pattern through both paths (staged twice, then from the
        direct slot when available) and agree on the outcome across ranks; raise when any rank
        saw a mismatch."""
        dev = torch.device("cuda", self.device)
        ok = 1
        n = 4099 * 4  # odd count of 16-B vectors (exercises the grid-stride tails)
        for salt in (1, 2, 3):
            pat = (torch.arange(n, device=dev, dtype=torch.int32) * (self.rank + 7) + salt * 1000003)
            inp = pat
            if salt == 3:  # direct slot: assembled in place, read by the peers from slot D
                if not self._direct_ok:
                    break
                inp = self._x.slot_tensor(n * 4).view(torch.int32)
                inp.copy_(pat)
            got = torch.empty(self.world_size * n, dtype=torch.int32, device=dev)
            ref = torch.empty_like(got)
            # the one-shot path itself, whatever a probe would pick for this size: the
            # self-check must never compare the inner comm against itself
            self._one_shot(got, inp, None)
            self.inner.all_gather_into(ref, pat).wait()
            torch.cuda.synchronize(dev)
            ok &= int(torch.equal(got, ref)) & int(_health.status()[1] == 0)
        # the one-shot all-to-all (QSGD's compressed-domain reduce-scatter) against the inner comm
        if self.world_size > 1:
            m = 16 * self.world_size * 131  # int32 words: W chunks of 16-B granular size
            pat = torch.arange(m, device=dev, dtype=torch.int32) * (self.rank + 5) + 11
            got, ref = torch.empty_like(pat), torch.empty_like(pat)
            self._a2a(got, pat)
            self.inner.all_to_all(ref, pat).wait()
            torch.cuda.synchronize(dev)
            ok &= int(torch.equal(got, ref)) & int(_health.status()[1] == 0)
        self._agree(bool(ok), "xGMI one-shot collectives failed their self-check against the inner comm")
        self.one_shot_calls = self.direct_calls = 0

    def _all(self, flag: bool) -> bool:
        """True on every rank iff ``flag`` is true on every rank."""
        dev = torch.device("cuda", self.device)
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
        self.inner.all_reduce(t, "min").wait()
        torch.cuda.synchronize(dev)
        return int(t.item()) == 1

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
