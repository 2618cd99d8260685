"""RandomKCompressor -- send k = max(1, int(n * ratio)) randomly chosen entries per tensor.

Reference: /root/reference/grace_dl/dist/compressor/randomk.py:6-40.  Indices are never sent:
every rank derives the same ones from (name, step).  Differences by design (survey 2.14 #8):

* the reference reseeds the GLOBAL torch RNG (``torch.manual_seed``) on every call, changing
  dropout / QSGD / weight-init randomness as a side effect; here indices come from a private
  keyed Feistel permutation (csrc/include/grace_rand.h) -- O(1) per index instead of a full
  ``randperm(n)``;
* the step counter is kept per name (not one global counter), so ranks agree even if they
  compress buckets in different orders (DDP bucket readiness order).

Payload: [vals fp32 (K)].  Allreduce-compatible (identical indices on every rank).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import torch

from ..core import Compressor, layout_of
from ._base import StepState
from ..memory.residual import ResidualMemory
from ..ops import randomk as R
from ..ops.elementwise import axpby
from ..ops.layout import SegmentLayout
from ..ops.topk import k_per_segment
from ..parallel.comm import stack_rows


@dataclass
class RandomKCtx:
    layout: SegmentLayout
    ks: Tuple[int, ...]
    seeds: Tuple[int, ...]
    numel: int
    shape: torch.Size
    dtype: torch.dtype
    step: int = 0                      # host step (mixed into the seeds on the torch path)
    step_t: Optional[torch.Tensor] = None  # device step counter (mixed in by the kernels)


class RandomKCompressor(StepState, Compressor):
    allreduce_compatible = True
    _state_attrs = ("steps",)

    def __init__(self, compress_ratio: float, seed: int = 0):
        super().__init__()
        self.compress_ratio = compress_ratio
        self.seed = seed
        self._init_steps()

    @property
    def global_step(self) -> int:  # reference attribute name
        return sum(self.steps.values())

    def _ctx(self, tensor, name) -> RandomKCtx:
        lay = layout_of(tensor, name)
        ks = k_per_segment(lay, self.compress_ratio)
        step, step_t = self.advance(name, tensor.device)
        # per-segment base seeds are step-independent; the step is mixed in by R.gather/scatter
        # (on device when step_t is given, so graph replays draw new indices)
        base = R.fnv1a64(name.encode("utf8")) ^ (self.seed * 0x9E3779B97F4A7C15 & 0xFFFFFFFFFFFFFFFF)
        seeds = tuple((base ^ (0xBF58476D1CE4E5B9 * (i + 1))) & 0xFFFFFFFFFFFFFFFF for i in range(lay.n_seg))
        return RandomKCtx(lay, ks, seeds, tensor.numel(), tensor.shape, tensor.dtype, step, step_t)

    def compress(self, tensor, name):
        ctx = self._ctx(tensor, name)
        x = tensor.reshape(-1).float().contiguous()
        vals = R.gather(x, ctx.layout, ctx.ks, ctx.seeds, step=ctx.step, step_t=ctx.step_t)
        return [vals], ctx

    def fused_compress(self, tensor, name, memory):
        if not isinstance(memory, ResidualMemory):
            return None
        ctx = self._ctx(tensor, name)
        g = tensor.reshape(-1).float().contiguous()
        r, valid = memory.residual_buffer(name, g)
        if valid:
            axpby(r, g, memory.beta, memory.gamma, out=r)
        else:
            r.copy_(g)
        # gather the sent values and zero them in the residual in the same kernel
        vals = R.gather(r, ctx.layout, ctx.ks, ctx.seeds, zero_selected=True, step=ctx.step, step_t=ctx.step_t)
        return [vals], ctx

    def _scale(self, world_size: int) -> float:
        return 1.0 / world_size if self.average else 1.0

    def indices(self, ctx: RandomKCtx, device="cpu") -> torch.Tensor:
        return R.indices(ctx.layout, ctx.ks, ctx.seeds, device, step=ctx.step)

    def decompress(self, tensors, ctx):
        (vals,) = tensors
        out = torch.zeros(ctx.numel, dtype=torch.float32, device=vals.device)
        R.scatter(vals, ctx.layout, ctx.ks, ctx.seeds, out, 1.0, step=ctx.step, step_t=ctx.step_t)
        return out.view(ctx.shape).to(ctx.dtype)

    def decompress_reduced(self, tensors, ctx, world_size):
        (vals,) = tensors
        out = torch.zeros(ctx.numel, dtype=torch.float32, device=vals.device)
        R.scatter(vals, ctx.layout, ctx.ks, ctx.seeds, out, self._scale(world_size),
                  step=ctx.step, step_t=ctx.step_t)
        return out.view(ctx.shape).to(ctx.dtype)

    def decompress_aggregate(self, per_rank, ctx, world_size):
        rows = stack_rows([p[0] for p in per_rank])
        out = torch.zeros(ctx.numel, dtype=torch.float32, device=rows.device)
        R.scatter(rows, ctx.layout, ctx.ks, ctx.seeds, out, self._scale(world_size),
                  step=ctx.step, step_t=ctx.step_t)
        return out.view(ctx.shape).to(ctx.dtype)
