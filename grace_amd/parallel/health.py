"""Process-wide communication health (csrc/comm/health.cpp).

Device kernels that can detect a communication fault (the xGMI one-shot all-gather's bounded
peer waits) raise a flag in two places: device memory, which ``FusedSGD``'s kernel reads so it
skips the update of that step (a corrupted exchange never reaches the weights, also inside a
replayed HIP graph), and pinned host-mapped memory, which :func:`check` reads with a plain load --
no device synchronisation, safe while a stream is being captured, cheap enough for every step.
The reference's only failure signal is Horovod's handle table
(/root/reference/patch_files/horovod/torch/mpi_ops.py:407-439).
"""
from __future__ import annotations

from typing import Tuple

import torch

from ..ops import _native


class CommFault(RuntimeError):
    """A device-side communication fault (peer wait timed out, ...)."""


_INIT = False
_DEVICES = set()


def init(device=None) -> bool:
    """Allocate the health words (before any graph capture): the process-wide host-mapped words
    once, and the fault word of ``device`` (default: the current device) -- each device's
    optimizer / comm kernels only touch their own device's word.  False off the GPU path."""
    global _INIT
    if not (torch.cuda.is_available() and _native.available()):
        return False
    if isinstance(device, int):
        idx = device
    elif device is not None and torch.device(device).index is not None:
        idx = torch.device(device).index
    else:
        idx = torch.cuda.current_device()
    if idx not in _DEVICES:
        _native.lib().health_init(int(idx))
        _DEVICES.add(idx)
    _INIT = True
    return True


def init_for(t: torch.Tensor) -> None:
    """``init(t.device)`` for a GPU tensor, once per device; a no-op while a stream is being
    captured (allocation is for the eager steps before a capture)."""
    if t.is_cuda and t.device.index not in _DEVICES and not torch.cuda.is_current_stream_capturing():
        init(t.device)


def status() -> Tuple[int, int]:
    """(fault flag, xGMI peer-wait timeouts) -- host-mapped read, no sync."""
    if not _INIT:
        return 0, 0
    f, t = _native.lib().health_check()[:2]
    return int(f), int(t)


def overflows() -> int:
    """Capacity payloads whose selection did not fit since the last reset (Threshold / DGC
    spill into the residual; INCEPTIONN with a capacity < 1 drops classes) -- counted by the
    kernels on the device, so steps replayed from a HIP graph are included.  Host-mapped read."""
    if not _INIT:
        return 0
    return int(_native.lib().health_check()[2])


def check() -> None:
    f, t = status()
    if f:
        raise CommFault(f"communication fault on the device ({t} xGMI peer wait(s) timed out): the optimizer "
                        "skipped its update; a peer died or diverged")


def reset() -> None:
    if _INIT:
        _native.lib().health_reset()
