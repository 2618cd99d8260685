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


def init() -> bool:
    """Allocate the health words (before any graph capture).  False off the GPU path."""
    global _INIT
    if _INIT:
        return True
    if not (torch.cuda.is_available() and _native.available()):
        return False
    _native.lib().health_init()
    _INIT = True
    return True


def status() -> Tuple[int, int]:
    """(fault flag, xGMI peer-wait timeouts) -- host-mapped read, no sync."""
    if not _INIT:
        return 0, 0
    f, t = _native.lib().health_check()
    return int(f), int(t)


def check() -> None:
    f, t = status()
    if f:
        raise CommFault(f"communication fault on the device ({t} xGMI peer wait(s) timed out): the optimizer "
                        "skipped its update; a peer died or diverged")


def reset() -> None:
    if _INIT:
        _native.lib().health_reset()
