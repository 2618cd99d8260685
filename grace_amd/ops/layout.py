"""Segment layouts: how a flat gradient bucket is split into parameter tensors.

The reference compresses one parameter tensor at a time
(/root/reference/examples/dist/CIFAR10-dawndist/core.py:203-206 and
/root/reference/patch_files/horovod/torch/__init__.py:124-141).  grace_amd keeps the
*per-tensor semantics* (e.g. Top-K keeps k_i = max(1, int(n_i * ratio)) per tensor) but
executes whole buckets in single kernel launches.  A :class:`SegmentLayout` carries

* ``offsets``  - flat start of each segment (len n_seg + 1, host ints)
* ``shapes``   - original tensor shapes (for per-tensor decompress / PowerSGD matrices)
* a device *chunk table* - (segment id, begin, end) for work chunks that never straddle a
  segment, so a workgroup knows its segment with no search.  Chunk size is chosen so that a
  bucket yields >> 256 workgroups (MI355X has 256 CUs).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

import torch

DEFAULT_CHUNK = 8192


@dataclass
class SegmentLayout:
    numels: Tuple[int, ...]
    shapes: Tuple[Tuple[int, ...], ...]
    chunk: int = DEFAULT_CHUNK
    offsets: Tuple[int, ...] = field(init=False)
    _dev: Dict[str, dict] = field(default_factory=dict, init=False, repr=False)

    def __post_init__(self):
        offs = [0]
        for n in self.numels:
            offs.append(offs[-1] + int(n))
        self.offsets = tuple(offs)

    # ------------------------------------------------------------------ constructors
    @classmethod
    def from_tensors(cls, tensors: Sequence[torch.Tensor], chunk: int = DEFAULT_CHUNK) -> "SegmentLayout":
        return cls(tuple(int(t.numel()) for t in tensors), tuple(tuple(t.shape) for t in tensors), chunk)

    @classmethod
    def single(cls, t: torch.Tensor, chunk: int = DEFAULT_CHUNK) -> "SegmentLayout":
        return cls((int(t.numel()),), (tuple(t.shape),), chunk)

    # ------------------------------------------------------------------ properties
    @property
    def n_seg(self) -> int:
        return len(self.numels)

    @property
    def total(self) -> int:
        return self.offsets[-1]

    def segments(self):
        for i, n in enumerate(self.numels):
            yield i, self.offsets[i], n

    def word_offsets(self) -> List[int]:
        """Per-segment offsets of 64-element groups (1 uint64 bit-plane word per group)."""
        w = [0]
        for n in self.numels:
            w.append(w[-1] + (n + 63) // 64)
        return w

    @property
    def n_words(self) -> int:
        return self.word_offsets()[-1]

    def views(self, flat: torch.Tensor) -> List[torch.Tensor]:
        return [flat[o:o + n].view(s) for (_, o, n), s in zip(self.segments(), self.shapes)]

    # ------------------------------------------------------------------ chunk table
    def _host_chunks(self, chunk: int):
        seg, beg, end = [], [], []
        for i, o, n in self.segments():
            if n == 0:
                continue
            nch = max(1, math.ceil(n / chunk))
            for c in range(nch):
                b = o + c * chunk
                seg.append(i)
                beg.append(b)
                end.append(min(o + n, b + chunk))
        return seg, beg, end

    def device_tables(self, device: torch.device, chunk: int | None = None) -> dict:
        """Device-resident chunk table (cached per device/chunk size)."""
        chunk = chunk or self.chunk
        key = f"{device}:{chunk}"
        d = self._dev.get(key)
        if d is None:
            seg, beg, end = self._host_chunks(chunk)
            scb = [0] * (self.n_seg + 1)
            for s_ in seg:
                scb[s_ + 1] += 1
            for i in range(self.n_seg):
                scb[i + 1] += scb[i]
            d = {
                "seg_chunk_begin": torch.tensor(scb, dtype=torch.int32, device=device),
                "seg": torch.tensor(seg, dtype=torch.int32, device=device),
                "begin": torch.tensor(beg, dtype=torch.int64, device=device),
                "end": torch.tensor(end, dtype=torch.int64, device=device),
                "offsets": torch.tensor(self.offsets, dtype=torch.int64, device=device),
                "n_chunks": len(seg),
                "word_off": torch.tensor(self.word_offsets(), dtype=torch.int64, device=device),
            }
            self._dev[key] = d
        return d

    def cached(self, device: torch.device, name: str, builder):
        """Per-layout cache of derived device tensors (k per segment, workspaces, ...)."""
        key = f"{device}:{name}"
        v = self._dev.get(key)
        if v is None:
            v = builder()
            self._dev[key] = v
        return v

    def numels_t(self, device, dtype=torch.float32) -> torch.Tensor:
        """Segment sizes as a cached device tensor (no per-step host->device copy, so code
        using it can run inside a HIP-graph capture)."""
        return self.cached(device, f"numels:{dtype}", lambda: torch.tensor(self.numels, dtype=dtype, device=device))

    def offsets_t(self, device, dtype=torch.int64) -> torch.Tensor:
        return self.cached(device, f"offsets:{dtype}", lambda: torch.tensor(self.offsets, dtype=dtype, device=device))


_LAYOUT_CACHE: Dict[Tuple, SegmentLayout] = {}


def layout_for(tensors_or_shapes, chunk: int = DEFAULT_CHUNK) -> SegmentLayout:
    """Interned layout for a sequence of tensors (or shapes)."""
    shapes = tuple(tuple(t.shape) if isinstance(t, torch.Tensor) else tuple(t) for t in tensors_or_shapes)
    key = (shapes, chunk)
    lay = _LAYOUT_CACHE.get(key)
    if lay is None:
        numels = tuple(int(math.prod(s)) if len(s) else 1 for s in shapes)
        lay = SegmentLayout(numels, shapes, chunk)
        _LAYOUT_CACHE[key] = lay
    return lay
