"""Fixed-capacity sparse payloads with an in-band count (the variable-size codecs' wire format).

The reference exchanges variable-size payloads by first all-gathering the sizes, reading them on
the host and padding every tensor to the maximum (/root/reference/grace_dl/dist/communicator/
allgather.py:15-38; the Horovod variant blocks inside the backward hook,
grace_dl/torch/communicator/allgather.py:27-30).  That is a host round trip per tensor and
makes the step impossible to capture in a HIP graph.

Here a variable-size codec (Threshold, DGC, Adaq, INCEPTIONN) writes into a payload of FIXED
capacity whose first 16 bytes are an int32 header ``[selected, capacity, 0, 0]`` filled on the
device by the compaction kernel.  Every rank's payload has the same byte size, so the Allgather /
Broadcast communicators take their same-size path (one packed collective, no size exchange), and
the decoders read ``min(selected, capacity)`` from each rank's header on the device.  Entries
selected beyond the capacity are not sent; with an error-feedback memory they stay in the
residual and go out in a later step (spill, not loss).  ``selected > capacity`` is visible in
the header (``overflow``) for monitoring.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch

from . import _native

HEADER_WORDS = 4


def capacity(n: int, ratio: float) -> int:
    """Entries of a payload for ``n`` candidates at capacity ``ratio`` (1.0 = exact, never spills)."""
    return max(1, min(int(n), int(math.ceil(ratio * n)))) if n > 0 else 1


def sparse_payload(device, cap: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """(header int32[4], values fp32[cap], indices int32[cap]) as views of ONE wire buffer."""
    from ..parallel.comm import PayloadBuilder

    hdr, v, i = PayloadBuilder(device, [(torch.int32, (HEADER_WORDS,)), (torch.float32, (cap,)),
                                        (torch.int32, (cap,))]).tensors
    return hdr, v, i


def scatter_capped(hdr: torch.Tensor, vals: torch.Tensor, idx: torch.Tensor, out: torch.Tensor,
                   scale: float = 1.0, accumulate: bool = True) -> None:
    """out[idx[j]] (+)= vals[j] * scale for j < min(hdr[0], capacity) -- the count is read on the
    device on the native path (no host sync)."""
    if _native.use_native(out):
        _native.lib().sparse_scatter_add_dev(vals, idx, hdr[:1], out, scale, accumulate)
        return
    k = min(int(hdr[0]), vals.numel())
    il = idx[:k].long()
    if accumulate:
        out.index_add_(0, il, vals[:k] * scale)
    else:
        out[il] = vals[:k] * scale


def zero_capped(hdr: torch.Tensor, idx: torch.Tensor, out: torch.Tensor, zeros: torch.Tensor) -> None:
    """out[idx[j]] = 0 for the sent entries (``zeros``: a cached all-zero fp32 buffer >= capacity)."""
    scatter_capped(hdr, zeros[: idx.numel()], idx, out, 1.0, accumulate=False)


def sent(hdr: torch.Tensor, cap: int) -> int:
    """Host-side count of the sent entries (monitoring / tests only: a device->host read)."""
    return min(int(hdr[0]), cap)


def overflow(hdr: torch.Tensor, cap: int) -> bool:
    return int(hdr[0]) > cap
