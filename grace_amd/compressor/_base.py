"""Shared plumbing for the bucket-aware compressors."""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Tuple

import torch

from ..core import Compressor, layout_of
from ..ops import _native
from ..ops.layout import SegmentLayout
from ..ops.randomk import fnv1a64, mix_step
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


class DeviceSteps:
    """Per-name step counters mirrored in device memory.

    A stochastic codec's kernel reads its step from a 1-element int64 device tensor and mixes it
    into the Philox / Feistel seed (``csrc/include/grace_common.h`` SeedArg).  ``bump`` issues an
    ``add_(1)`` on the current stream, so a HIP-graph replay of the step advances the counter
    too: the randomness stays fresh on every replay instead of freezing the capture-time seed.
    In eager mode the device value always equals the host counter ``steps[name]``.
    """

    def __init__(self):
        self._t: Dict[str, torch.Tensor] = {}
        self._post: set = set()

    def bump(self, name: str, device: torch.device, host_value: int, post: bool = False) -> torch.Tensor:
        """``post=True``: the caller's kernel advances the counter itself AFTER its readers ran
        (PowerSGD's P = M Q launch, one launch fewer than the ``add_``): the counter is created
        at ``host_value`` and not advanced here, and holds step + 1 between steps."""
        t = self._t.get(name)
        if t is None or t.device != device or (name in self._post) != post:
            t = torch.full((1,), host_value, dtype=torch.int64, device=device)
            self._t[name] = t
            (self._post.add if post else self._post.discard)(name)
        elif not post:
            t.add_(1)
        return t

    def sync_to(self, steps: Dict[str, int]) -> None:
        """Copy the device counters (advanced by graph replays) back into the host dict."""
        for name, t in self._t.items():
            steps[name] = int(t.item()) - (1 if name in self._post else 0)

    def reset(self) -> None:
        self._t.clear()
        self._post.clear()


class StepState:
    """Mixin: host ``steps`` dict + device mirrors, kept consistent through state_dict."""

    def _init_steps(self):
        self.steps: Dict[str, int] = {}
        self._dsteps = DeviceSteps()

    def advance(self, name: str, device, post: bool = False) -> Tuple[int, Any]:
        """Advance ``name``'s step.  Returns (host step, device counter or None); ``post``: see
        :meth:`DeviceSteps.bump` (the caller MUST advance the device counter after using it)."""
        step = self.steps.get(name, 0) + 1
        self.steps[name] = step
        if _native.native_on(device):
            return step, self._dsteps.bump(name, torch.device(device), step, post=post)
        return step, None

    def state_dict(self):
        self._dsteps.sync_to(self.steps)
        return super().state_dict()

    def load_state_dict(self, state):
        super().load_state_dict(state)
        self._dsteps.reset()


class BucketCompressor(StepState, Compressor):
    """Compressor whose kernels run over a whole flat bucket (per-segment semantics)."""

    _state_attrs: Tuple[str, ...] = ("steps",)

    def __init__(self, average=True, tensors_size_are_same=True):
        super().__init__(average, tensors_size_are_same)
        self._init_steps()
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

    def base_seed(self, name: str) -> int:
        """Per-(name, rank) seed: independent rounding noise on every rank."""
        return (fnv1a64(name.encode("utf8")) ^ (0xD1B54A32D192ED03 * (self.rank + 1))) & MASK64

    def next_seed(self, name: str) -> int:
        """Per-(name, step, rank) host seed (for codecs without a device step counter)."""
        step, _ = self.advance(name, "cpu")
        return mix_step(self.base_seed(name), step)

    def next_rng(self, name: str, device):
        """(seed, step_tensor) for a native kernel: the kernel mixes the DEVICE step into the
        seed (graph-replay safe).  Off the native path: (host-mixed seed, None)."""
        step, t = self.advance(name, device)
        if t is None:
            return mix_step(self.base_seed(name), step), None
        return self.base_seed(name), t

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
