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
                   scale: float = 1.0, accumulate: bool = True, count_overflow: bool = False) -> None:
    """out[idx[j]] (+)= vals[j] * scale for j < min(hdr[0], capacity) -- the count is read on the
    device on the native path (no host sync).  ``count_overflow``: this is the decode of the
    process's OWN payload, so an overflow (hdr[0] > capacity) is counted in health.overflows() --
    once per overflowing payload, not once per rank that decodes it."""
    if _native.use_native(out):
        _native.lib().sparse_scatter_add_dev(vals, idx, hdr[:1], out, scale, accumulate, count_overflow)
        return
    k = min(int(hdr[0]), vals.numel())
    il = idx[:k].long()
    if accumulate:
        out.index_add_(0, il, vals[:k] * scale)
    else:
        out[il] = vals[:k] * scale


def set_own_rank(ctx, rank) -> None:
    """Record the decoding process's rank on a compress ctx (the communicators do, before the
    decode): the decoders count capacity overflows for that payload only."""
    if rank is None:
        return
    try:
        ctx.own_rank = int(rank)
    except (AttributeError, TypeError):  # a ctx that takes no attributes (tuple / slots): not counted
        pass


def own_rank(ctx):
    """The decoding process's rank recorded by ``set_own_rank`` (None: unknown, then no overflow
    is counted by the decode)."""
    return getattr(ctx, "own_rank", None)


def decode_ranks(vals, idxs, counts, out: torch.Tensor, scale: float = 1.0, own=None) -> torch.Tensor:
    """``out`` = 0, then ``out[idxs[r]] += vals[r] * scale`` for r = 0..W-1 in rank order --
    bit-identical on every rank.  ``counts[r]``: None (every entry) or the payload's in-band count
    word (capacity payloads: the first min(count, capacity) entries).  Native path: a zero fill plus
    W atomic-free scatter launches.  (A one-launch form -- zero + W rank phases behind grid barriers
    -- was measured in round 4: as fast stand-alone, 51 vs ~28 us inside the whole-step graph where
    its barriers wait on workgroups sharing the chip with side-stream weight gradients; deleted.)
    ``own``: this process's rank -- only that payload's overflow is counted (health.overflows())."""
    out.zero_()
    native = _native.use_native(out)
    for r, (v, i, c) in enumerate(zip(vals, idxs, counts)):  # fixed rank order: identical on every rank
        if c is not None:
            scatter_capped(c, v, i, out, scale, accumulate=True, count_overflow=(r == own))
        elif native:
            _native.lib().sparse_scatter_add(v, i, out, scale, True)
        else:
            out.index_add_(0, i.long(), v * scale)
    return out


def zero_capped(hdr: torch.Tensor, idx: torch.Tensor, out: torch.Tensor, zeros: torch.Tensor) -> None:
    """out[idx[j]] = 0 for the sent entries (``zeros``: a cached all-zero fp32 buffer >= capacity)."""
    scatter_capped(hdr, zeros[: idx.numel()], idx, out, 1.0, accumulate=False)


def sent(hdr: torch.Tensor, cap: int) -> int:
    """Host-side count of the sent entries (monitoring / tests only: a device->host read)."""
    return min(int(hdr[0]), cap)


def overflow(hdr: torch.Tensor, cap: int) -> bool:
    return int(hdr[0]) > cap


class AdaptiveCapacity:
    """Per-name payload capacity: starts at ``ratio`` of the tensor and GROWS (never shrinks)
    when a step's in-band count shows the payload overflowed -- with no host synchronisation.

    After each exchange the count words of EVERY rank's header (the gathered payloads: the same
    bytes on every rank) are reduced to their max on the device and copied to pinned host memory
    by a non-blocking copy (``observe``); the host reads that at the NEXT compress of the same
    name, after waiting on the copy's event (recorded a whole step earlier: no real stall).  So
    every rank takes the same decision at the same step and the payloads stay equal-sized.  When
    the need exceeded the capacity the capacity becomes ``grow`` x the need (<= the tensor).
    Nothing adapts while a stream is being captured: a captured HIP graph keeps the capacity it
    was captured with (its payload buffers are static), and entries past it spill -- into the
    residual when an error-feedback memory is fused (no loss), or are dropped (counted in
    ``overflow_steps``).  SURVEY 2.11: the reference pads to the max actual size instead, with a
    size all-gather and a host read per tensor (grace_dl/dist/communicator/allgather.py:15-38).
    """

    def __init__(self, ratio: float, grow: float = 1.5):
        self.ratio = float(ratio)
        self.grow = float(grow)
        self.cap = {}        # name -> entries (or bytes, as the codec defines its unit)
        self._probe = {}     # name -> (pinned int32 words, event, need_fn)
        self.overflow_steps = 0

    def get(self, name: str, n: int, unit_max: int) -> int:
        """Current capacity of ``name`` (initially ceil(ratio * n), clamped to [1, unit_max])."""
        self._poll(name, unit_max)
        c = self.cap.get(name)
        if c is None:
            c = max(1, min(int(unit_max), int(math.ceil(self.ratio * n))))
            self.cap[name] = c
        return c

    def _poll(self, name: str, unit_max: int) -> None:
        pr = self._probe.get(name)
        if pr is None or _capturing():  # no host wait inside a capture: the probe waits for an eager step
            return
        words, ev, need_fn = pr
        if ev is not None:
            ev.synchronize()  # recorded one step ago; a deterministic step for every rank
        del self._probe[name]
        need = int(need_fn([int(w) for w in words.tolist()]))
        cur = self.cap.get(name, 0)
        if need > cur:
            self.overflow_steps += 1
            if not _capturing():
                self.cap[name] = max(cur, min(int(unit_max), int(math.ceil(self.grow * need))))

    def observe(self, name: str, headers, need_fn) -> None:
        """Queue a lagged read of the element-wise max over ``headers`` (every rank's int32 count
        words, identical on all ranks); ``need_fn(words) -> units needed``."""
        if _capturing():
            return
        hdr = headers[0] if len(headers) == 1 else torch.stack([h.reshape(-1) for h in headers]).amax(0)
        if hdr.is_cuda:
            words = torch.empty(hdr.numel(), dtype=torch.int32, pin_memory=True)
            words.copy_(hdr, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            words, ev = hdr.clone(), None
        self._probe[name] = (words, ev, need_fn)


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
