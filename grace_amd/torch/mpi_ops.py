"""Horovod-style collective API over the grace_amd comm layer (RCCL on MI355X, gloo on CPU).

Mirrors the surface of the reference's patched ``horovod.torch.mpi_ops``
(/root/reference/patch_files/horovod/torch/mpi_ops.py:57-439): ``allreduce[_][_async]``,
``allgather[_async]``, ``broadcast[_][_async]``, ``poll`` and ``synchronize`` on integer handles
kept in a handle table that holds the input/output tensors alive until synchronised
(mpi_ops.py:57-60), plus ``init/size/rank/local_rank``.

Design differences (MI355X-first):
* no background thread / negotiation: a handle wraps the comm layer's async ``Work`` (RCCL
  runs on its own stream; ``synchronize`` is a stream-level wait, the host never blocks);
* one dtype-generic path instead of per-dtype C entry points (mpi_ops.py:66-89);
* ``allgather`` supports a different first dimension per rank like Horovod (sizes are
  exchanged once with a tiny allgather, then one padded all-gather of the payload);
* averaging divides in place after the reduction (Horovod's ``average=True``).
"""
from __future__ import annotations

import itertools
import os
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..parallel import comm as _comm

_handles: Dict[int, Tuple] = {}
_next = itertools.count(1)


# ------------------------------------------------------------------------------ process info
def init(backend: Optional[str] = None) -> None:
    """Initialise torch.distributed from the torchrun environment (idempotent) and pin the GPU."""
    if not dist.is_initialized():
        from ..parallel.launch import init_distributed

        init_distributed(backend=backend)


def is_initialized() -> bool:
    return dist.is_initialized()


def shutdown() -> None:
    _handles.clear()
    if dist.is_initialized():
        dist.destroy_process_group()
    _comm.set_default_comm(None)


def size() -> int:
    return _comm.default_comm().world_size


def rank() -> int:
    return _comm.default_comm().rank


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def local_size() -> int:
    return int(os.environ.get("LOCAL_WORLD_SIZE", str(size())))


# ------------------------------------------------------------------------------ handles
def _register(work, output, post=None) -> int:
    h = next(_next)
    _handles[h] = (work, output, post)
    return h


def poll(handle: int) -> bool:
    """True when the collective behind ``handle`` has completed (never blocks)."""
    if handle not in _handles:
        raise ValueError(f"unknown handle {handle}")
    return _handles[handle][0].is_completed()


def synchronize(handle: int) -> torch.Tensor:
    """Wait for ``handle`` (stream-level for GPU tensors) and return its output tensor."""
    if handle not in _handles:
        raise ValueError(f"unknown handle {handle}")
    work, output, post = _handles.pop(handle)
    work.wait()
    return post(output) if post is not None else output


# ------------------------------------------------------------------------------ allreduce
def allreduce_async_(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None) -> int:
    c = _comm.default_comm()
    w = c.all_reduce(tensor, "sum", async_op=True)
    n = c.world_size

    def post(t):
        if average and n > 1:
            if t.is_floating_point():
                t.div_(n)
            else:
                t.floor_divide_(n)
        return t

    return _register(w, tensor, post)


def allreduce_async(tensor: torch.Tensor, average: bool = True, name: Optional[str] = None) -> int:
    return allreduce_async_(tensor.clone(), average, name)


def allreduce_(tensor, average=True, name=None):
    return synchronize(allreduce_async_(tensor, average, name))


def allreduce(tensor, average=True, name=None):
    return synchronize(allreduce_async(tensor, average, name))


# ------------------------------------------------------------------------------ allgather
def allgather_async(tensor: torch.Tensor, name: Optional[str] = None) -> int:
    """Concatenate every rank's ``tensor`` along dim 0 (first dims may differ per rank)."""
    work, finish = _comm.allgather_rows(_comm.default_comm(), tensor, async_op=True)
    return _register(work, None, lambda _: finish())


def allgather(tensor, name=None):
    return synchronize(allgather_async(tensor, name))


# ------------------------------------------------------------------------------ broadcast
def broadcast_async_(tensor: torch.Tensor, root_rank: int, name: Optional[str] = None) -> int:
    w = _comm.default_comm().broadcast(tensor, root_rank, async_op=True)
    return _register(w, tensor)


def broadcast_async(tensor: torch.Tensor, root_rank: int, name: Optional[str] = None) -> int:
    return broadcast_async_(tensor.clone(), root_rank, name)


def broadcast_(tensor, root_rank, name=None):
    return synchronize(broadcast_async_(tensor, root_rank, name))


def broadcast(tensor, root_rank, name=None):
    return synchronize(broadcast_async(tensor, root_rank, name))
