"""Allreduce communicator.

Reference: /root/reference/grace_dl/dist/communicator/allreduce.py:6-13 (in-place SUM
all-reduce of every payload tensor, ``div_(W)`` when averaging, then one decompress) and the
async Horovod variant /root/reference/grace_dl/torch/communicator/allreduce.py:5-15.

Differences by design:
* every payload tensor of one dtype moves in ONE all-reduce (packed) instead of one each;
* the divide-by-W is done by the compressor's ``decompress_reduced`` so kernels can fuse it;
* pairs that are not linear under summation (reference compatibility matrix)
  are rejected up front instead of silently producing wrong gradients -- unless the
  compressor implements a compressed-domain reduction: QSGD switches to shared-scale integer
  levels (``enable_allreduce_mode``), sign/ternary/8-bit codecs reduce by all-gathering their
  bit-packed payload and decoding/voting all ranks in one kernel (``reduce_by_allgather``) --
  the all-reduce result, identical on every rank, with the fewest bytes on the xGMI links.
"""
from __future__ import annotations

from collections import OrderedDict

import torch

from ..core import Communicator
from .allgather import allgather_send, allgather_recv


class Allreduce(Communicator):
    def __init__(self, compressor, memory, world_size=None, comm=None, strict: bool = True):
        super().__init__(compressor, memory, world_size, comm)
        if hasattr(compressor, "enable_allreduce_mode"):
            compressor.enable_allreduce_mode()  # e.g. QSGD shared-scale integer levels
        # non-linear codecs reduce in the compressed domain: all-gather + one-pass decode/vote
        self._via_allgather = bool(getattr(compressor, "reduce_by_allgather", False))
        if strict and not getattr(compressor, "allreduce_compatible", False):
            raise ValueError(
                f"{type(compressor).__name__} payloads are not summable across ranks; use the Allgather "
                "or Broadcast communicator (or pass strict=False to reproduce the reference behaviour)")

    def async_send(self, tensors, name):
        if self._via_allgather:
            return ("ag", allgather_send(self.comm, self.compressor, tensors, self.world_size))
        rs = getattr(self.compressor, "rs_mode", None)
        if rs is not None and rs(self.world_size):  # QSGD: int8 all-to-all + int16 all-gather
            return ("rs", self.compressor.rs_send(self.comm, tensors[0]))
        tensors = list(tensors)
        works = []
        by_dtype = OrderedDict()
        for i, t in enumerate(tensors):
            by_dtype.setdefault(t.dtype, []).append(i)
        for dt, idxs in by_dtype.items():
            if len(idxs) == 1:
                t = tensors[idxs[0]]
                if not t.is_contiguous():
                    t = tensors[idxs[0]] = t.contiguous()
                works.append((self.comm.all_reduce(t, async_op=True), None, None))
            else:
                flat = torch.cat([tensors[i].reshape(-1) for i in idxs])
                works.append((self.comm.all_reduce(flat, async_op=True), flat, idxs))
        return ("ar", (tensors, works))

    def wait_comm(self, handles):
        kind, h = handles
        if kind == "rs":
            h[1].wait()
            return
        if kind == "ag":
            if h[3] is not None:
                h[3].wait()
            return
        for w, _, _ in h[1]:
            w.wait()

    def wait_receive(self, handles, ctx):
        kind, handles = handles
        if kind == "ag":
            return allgather_recv(handles, self.compressor, ctx, self.world_size, getattr(self.comm, "rank", None))
        if kind == "rs":
            return self.compressor.rs_receive(self.comm, handles, ctx, self.world_size)
        tensors, works = handles
        for w, flat, idxs in works:
            w.wait()
            if flat is not None:
                off = 0
                for i in idxs:
                    n = tensors[i].numel()
                    tensors[i] = flat[off:off + n].view_as(tensors[i])
                    off += n
        return self.compressor.decompress_reduced(tensors, ctx, self.world_size)
