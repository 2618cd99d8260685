"""Shared plumbing for the bucket-aware compressors."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Tuple

import torch

from ..core import Compressor, layout_of
from ..ops.layout import SegmentLayout
from ..ops.randomk import fnv1a64
from ..parallel.comm import PayloadBuilder, rank_rows

MASK64 = 0xFFFFFFFFFFFFFFFF


@dataclass
class Ctx:
    """Local context of one compress call (never sent)."""

    layout: SegmentLayout
    numel: int
    shape: torch.Size
    dtype: torch.dtype
    extra: Dict[str, Any] = field(default_factory=dict)
    #: optional destination for the aggregated result (the engine passes the bucket buffer so
    #: decompress writes the averaged gradient in place: no extra allocation / copy pass)
    out: Any = None


class BucketCompressor(Compressor):
    """Compressor whose kernels run over a whole flat bucket (per-segment semantics)."""

    _state_attrs: Tuple[str, ...] = ("steps",)

    def __init__(self, average=True, tensors_size_are_same=True):
        super().__init__(average, tensors_size_are_same)
        self.steps: Dict[str, int] = {}
        self.rank = 0

    def bind_comm(self, comm):
        self.comm = comm
        self.rank = comm.rank

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def flat(tensor: torch.Tensor) -> torch.Tensor:
        g = tensor.reshape(-1)
        if g.dtype != torch.float32:
            g = g.float()
        return g.contiguous()

    def ctx(self, tensor, name) -> Ctx:
        return Ctx(layout_of(tensor, name), tensor.numel(), tensor.shape, tensor.dtype)

    def next_seed(self, name: str) -> int:
        """Per-(name, step, rank) seed: independent rounding noise on every rank/step."""
        step = self.steps.get(name, 0)
        self.steps[name] = step + 1
        h = fnv1a64(name.encode("utf8"))
        return (h ^ (0x9E3779B97F4A7C15 * (step + 1)) ^ (0xD1B54A32D192ED03 * (self.rank + 1))) & MASK64

    @staticmethod
    def payload(device, entries):
        return PayloadBuilder(device, entries).tensors

    @staticmethod
    def rows(per_rank):
        return rank_rows(per_rank)

    @staticmethod
    def out_buffer(ctx, device, zero: bool = False) -> torch.Tensor:
        o = getattr(ctx, "out", None)
        if o is not None and o.device == device and o.dtype == torch.float32 and o.numel() == ctx.layout.total \
                and o.is_contiguous():
            ctx.out = None  # one use
            return o.view(-1).zero_() if zero else o.view(-1)
        return (torch.zeros if zero else torch.empty)(ctx.layout.total, dtype=torch.float32, device=device)

    def finish(self, out: torch.Tensor, ctx: Ctx) -> torch.Tensor:
        return out.view(ctx.shape).to(ctx.dtype) if ctx.dtype != torch.float32 else out.view(ctx.shape)

    def decompress(self, tensors, ctx):
        return self.decompress_aggregate_impl([list(tensors)], ctx, 1, 1.0)

    def decompress_aggregate(self, per_rank, ctx, world_size):
        scale = self.aggregate_scale(world_size)
        return self.decompress_aggregate_impl(per_rank, ctx, len(per_rank), scale)

    def aggregate_scale(self, world_size: int) -> float:
        return 1.0 / world_size if self.average else 1.0

    def decompress_aggregate_impl(self, per_rank, ctx, n_ranks: int, scale: float) -> torch.Tensor:
        raise NotImplementedError
