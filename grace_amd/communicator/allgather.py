"""Allgather communicator.

Reference: /root/reference/grace_dl/dist/communicator/allgather.py:7-45 and the async Horovod
variant /root/reference/grace_dl/torch/communicator/allgather.py:7-52:
all-gather every payload tensor (padding to the max size when ``tensors_size_are_same`` is
False, after an all-gather of the sizes), decompress each rank's payload, aggregate, divide by
W when averaging.

MI355X design:
* the whole payload (all tensors) is packed into ONE byte buffer -> ONE all-gather per
  call (RCCL over xGMI; with a bucket as the tensor that is one collective per bucket),
* the variable-size path exchanges the byte sizes with one tiny all-gather (device tensor of
  the payload's own device, not a hard-coded ``.cuda()`` as in the reference line 16),
* decompress + aggregate + average of the W payloads is one compressor call
  (``decompress_aggregate``) so kernels can do it in a single pass (rank-ordered sparse
  scatter for Top-K, popcount vote for signs, ...).
"""
from __future__ import annotations

import torch

from ..core import Communicator
from ..parallel.comm import pack, unpack


def allgather_send(comm, compressor, tensors, world_size):
    """Launch the (packed) all-gather of one payload; returns an opaque handle."""
    tensors = list(tensors)
    W = world_size
    if compressor.tensors_size_are_same:
        buf, specs = pack(tensors)
        out = torch.empty(W * buf.numel(), dtype=torch.uint8, device=buf.device)
        kw = {}
        if getattr(comm, "accepts_ranges", False) and buf.numel():
            var = compressor.wire_counts(tensors)
            if var is not None:  # count-aware transport: only the valid bytes of each peer move
                from ..parallel.xgmi import byte_ranges

                kw["ranges"] = byte_ranges(specs, var, buf.numel())
        work = comm.all_gather_into(out, buf, async_op=True, **kw) if buf.numel() else None
        return (out, buf.numel(), [specs] * W, work, buf)
    # variable size: exchange element counts, pad every tensor to the max over ranks
    dev = tensors[0].device
    counts = torch.tensor([t.numel() for t in tensors], dtype=torch.int64, device=dev)
    all_counts = torch.empty(W * counts.numel(), dtype=torch.int64, device=dev)
    comm.all_gather_into(all_counts, counts).wait()
    all_counts = all_counts.view(W, -1).cpu()  # host sync (same as the reference)
    maxc = all_counts.max(dim=0).values.tolist()
    padded = []
    for t, m in zip(tensors, maxc):
        t = t.reshape(-1)
        if t.numel() < m:
            p = torch.zeros(m, dtype=t.dtype, device=t.device)
            p[: t.numel()] = t
            t = p
        padded.append(t)
    buf, pspecs = pack(padded)
    out = torch.empty(W * buf.numel(), dtype=torch.uint8, device=dev)
    work = comm.all_gather_into(out, buf, async_op=True) if buf.numel() else None
    rank_specs = []
    for r in range(W):
        sp = []
        for s_, c in zip(pspecs, all_counts[r].tolist()):
            esz = torch.empty((), dtype=s_.dtype).element_size()
            sp.append(type(s_)(s_.dtype, (int(c),), s_.offset, int(c) * esz))
        rank_specs.append(sp)
    return (out, buf.numel(), rank_specs, work, buf)


def allgather_recv(handles, compressor, ctx, world_size, rank=None):
    out, span, rank_specs, work, _keep = handles
    if work is not None:
        work.wait()
    from ..ops.cappayload import set_own_rank

    set_own_rank(ctx, rank)  # the decoders count only this process's payload overflow
    per_rank = [unpack(out[r * span:(r + 1) * span], rank_specs[r]) for r in range(world_size)]
    return compressor.decompress_aggregate(per_rank, ctx, world_size)


class Allgather(Communicator):
    def async_send(self, tensors, name):
        return allgather_send(self.comm, self.compressor, tensors, self.world_size)

    def wait_comm(self, handles):
        if handles[3] is not None:
            handles[3].wait()

    def wait_receive(self, handles, ctx):
        return allgather_recv(handles, self.compressor, ctx, self.world_size, getattr(self.comm, "rank", None))
