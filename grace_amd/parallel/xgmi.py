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

* all-gathers whose per-rank payload fits the capacity (and is 16-B granular) run the two
  native launches on the CURRENT stream (graph-capturable, no host sync); everything else
  (all-reduce, broadcast, all-to-all, larger gathers) goes to ``inner``;
* construction exchanges HIP IPC handles through the torch.distributed Store and, by default,
  verifies one gather against ``inner`` (every rank must agree, else it raises and the caller
  keeps ``inner``);
* ``check()`` raises when a peer wait timed out (dead or diverged peer) -- the device never hangs.
"""
from __future__ import annotations

import itertools

import torch
import torch.distributed as dist

from . import comm as _comm
from ..ops import _native

_UID = itertools.count()


class XgmiComm(_comm.Comm):
    _c = None  # not an RcclComm: GroupedComm issues the deferred gathers through all_gather_into

    def __init__(self, inner: _comm.Comm, capacity_mb: float = 8.0, verify: bool = True, store=None):
        if not dist.is_initialized():
            raise RuntimeError("XgmiComm needs torch.distributed (its Store carries the IPC handles)")
        self.inner = inner
        self.rank, self.world_size = inner.rank, inner.world_size
        self.device = torch.cuda.current_device()
        self._x = _native.lib().XgmiPeers(self.rank, self.world_size, self.device, int(capacity_mb * 2 ** 20))
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

    def _fits(self, out: torch.Tensor, inp: torch.Tensor) -> bool:
        n = inp.numel() * inp.element_size()
        return (inp.is_cuda and out.is_cuda and n % 16 == 0 and 0 < n <= self.capacity
                and inp.is_contiguous() and out.is_contiguous()
                and inp.data_ptr() % 16 == 0 and out.data_ptr() % 16 == 0)

    def all_gather_into(self, out, inp, async_op=False):
        if not self._fits(out, inp):
            return self.inner.all_gather_into(out, inp, async_op)
        # stream-ordered on the current stream: complete for every later op on it
        self._x.all_gather(out.view(-1).view(torch.uint8), inp.view(-1).view(torch.uint8))
        self.one_shot_calls += 1
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
        t = int(self._x.timeouts())
        if t:
            raise RuntimeError(f"xGMI all-gather: {t} peer wait(s) timed out (a peer died or diverged)")
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
            ok &= int(torch.equal(got, ref)) & int(self._x.timeouts() == 0)
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
        self._x.close()
