"""Debug mode for the gradient exchange: race / divergence / NaN detection.

The reference has no sanitizers; its only guards are the Horovod optimizer assertions
(patch_files/horovod/torch/__init__.py:124-201).  grace_amd keeps those (engine/optimizer) and
adds an opt-in checker, enabled with ``GRACE_AMD_DEBUG=1`` or ``GraceEngine(debug=True)``:

* **phase barriers** -- the device is synchronised after the exchange of every bucket, so an
  asynchronous fault (bad index, illegal address) is reported at the bucket that caused it;
* **finiteness** -- every aggregated bucket must be finite (NaN/Inf name the bucket);
* **cross-rank bit identity** -- the data-parallel invariant: every rank must hold the SAME
  aggregated gradient bits.  A 64-bit checksum of each bucket is all-gathered and compared; a
  mismatch means a non-deterministic decompress, a stream race (buffer reused before the
  collective finished) or diverged compressor state.

It costs host syncs and one tiny collective per bucket: a debugging tool, not for benchmarks.
"""
from __future__ import annotations

import os
from typing import Optional

import torch


def enabled_from_env() -> bool:
    return os.environ.get("GRACE_AMD_DEBUG", "0") == "1"


def checksum(t: torch.Tensor) -> torch.Tensor:
    """Order-sensitive 64-bit checksum of the raw bits of ``t`` (int64 tensor of shape [1])."""
    bits = t.detach().contiguous().view(-1).view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    w = torch.arange(1, bits.numel() + 1, dtype=torch.int64, device=bits.device)
    return ((bits * (w * 2654435761 % 4294967291)).sum() & 0x7FFFFFFFFFFFFFFF).view(1)


class DivergenceError(RuntimeError):
    pass


class ExchangeChecker:
    def __init__(self, comm=None):
        self.comm = comm
        self.checked = 0

    def check_bucket(self, name: str, flat: torch.Tensor, step: Optional[int] = None) -> None:
        if flat.is_cuda:
            torch.cuda.synchronize(flat.device)  # surface async faults at this bucket
        if not torch.isfinite(flat).all():
            bad = int((~torch.isfinite(flat)).sum())
            raise FloatingPointError(f"{name}: {bad} non-finite values after the GRACE exchange")
        c = self.comm
        if c is not None and c.world_size > 1:
            mine = checksum(flat)
            allc = torch.empty(c.world_size, dtype=torch.int64, device=mine.device)
            c.all_gather_into(allc, mine)
            vals = allc.tolist()
            if len(set(vals)) != 1:
                raise DivergenceError(f"{name}: aggregated gradient differs across ranks "
                                      f"(checksums {vals}) -- data-parallel invariant broken")
        self.checked += 1
