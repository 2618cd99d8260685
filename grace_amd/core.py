"""GRACE core abstractions: Memory, Compressor, Communicator.

API parity with the reference's three roles
(/root/reference/grace_dl/dist/__init__.py:4-51 for torch.distributed and
/root/reference/grace_dl/torch/__init__.py:37-58 for the split-phase Horovod variant):

* ``Memory.compensate(tensor, name)`` / ``Memory.update(tensor, name, compressor, payload, ctx)``
* ``Compressor.compress(tensor, name) -> (payload_list, ctx)``, ``decompress(payload, ctx)``,
  ``aggregate(list)``; flags ``average`` and ``tensors_size_are_same``
* ``Communicator.step(tensor, name)`` = compensate -> compress -> update -> send_receive, and
  the split-phase ``send_step`` / ``receive_step`` used to overlap with backward.

MI355X-first extensions (all optional for user-written subclasses):

* ``Compressor.fused_compress(tensor, name, memory)``: one native pass that performs
  compensate + compress + residual update (e.g. Top-K + ResidualMemory).  Returns ``None`` when
  the (compressor, memory) pair has no fused kernel and the generic 3-call path runs.
* ``Compressor.decompress_aggregate(per_rank_payloads, ctx, world_size)``: decompress all W
  ranks' payloads and aggregate them in one native pass (e.g. popcount majority vote for signs,
  rank-ordered sparse scatter for Top-K) instead of W dense decompresses + a Python ``sum``.
* ``state_dict()`` / ``load_state_dict()`` on every component, so error-feedback residuals,
  momenta and RNG step counters survive checkpoint/resume (the reference never saves them).
* tensors may be whole flat *buckets*: a :class:`~grace_amd.ops.layout.SegmentLayout`
  registered under the bucket name keeps per-parameter semantics (see ``layout_of``).
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

from .ops.layout import SegmentLayout

# name -> SegmentLayout for flat buckets (registered by the engines in grace_amd.parallel)
_LAYOUTS: Dict[str, SegmentLayout] = {}


def register_layout(name: str, layout: SegmentLayout) -> None:
    _LAYOUTS[name] = layout


def layout_of(tensor: torch.Tensor, name: str) -> SegmentLayout:
    """Layout of ``tensor``: the registered bucket layout if ``name`` is a bucket, else one
    segment holding the whole tensor (reference per-tensor semantics)."""
    lay = _LAYOUTS.get(name)
    if lay is not None and lay.total == tensor.numel():
        return lay
    return SegmentLayout((int(tensor.numel()),), (tuple(tensor.shape),))


def _state_to(obj: Any, device=None):
    if isinstance(obj, torch.Tensor):
        return obj.detach().clone() if device is None else obj.detach().to(device, copy=True)
    if isinstance(obj, dict):
        return {k: _state_to(v, device) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_state_to(v, device) for v in obj)
    return obj


class Stateful:
    """state_dict support for the dict-of-tensors state every GRACE component keeps."""

    _state_attrs: Tuple[str, ...] = ()

    def state_dict(self) -> Dict[str, Any]:
        return {a: _state_to(getattr(self, a)) for a in self._state_attrs}

    def load_state_dict(self, state: Dict[str, Any]) -> None:
        for a in self._state_attrs:
            if a in state:
                cur = getattr(self, a)
                val = _state_to(state[a])
                if isinstance(cur, dict) and isinstance(val, dict):
                    cur.clear()
                    cur.update(val)
                else:
                    setattr(self, a, val)


class Memory(Stateful, ABC):
    """Error-feedback memory (reference dist/__init__.py:4-12)."""

    @abstractmethod
    def compensate(self, tensor: torch.Tensor, name: str) -> torch.Tensor:
        """Return the tensor corrected by the stored residual."""

    def update(self, tensor, name, compressor, tensors_compressed, ctx) -> None:
        """Update the residual after compression (default: no-op)."""


class Compressor(Stateful, ABC):
    """Compress / decompress / aggregate (reference dist/__init__.py:15-34)."""

    #: payload of every rank can be summed element-wise (valid for the Allreduce communicator)
    allreduce_compatible: bool = False

    def __init__(self, average: bool = True, tensors_size_are_same: bool = True):
        self.average = average
        self.tensors_size_are_same = tensors_size_are_same

    @abstractmethod
    def compress(self, tensor: torch.Tensor, name: str) -> Tuple[List[torch.Tensor], Any]:
        """Compress ``tensor``; returns (payload tensors, local context)."""

    @abstractmethod
    def decompress(self, tensors: Sequence[torch.Tensor], ctx: Any) -> torch.Tensor:
        """Inverse of compress for one rank's payload."""

    def aggregate(self, tensors: Sequence[torch.Tensor]) -> torch.Tensor:
        """Combine the decompressed tensors of all ranks (default: sum)."""
        out = tensors[0].clone()
        for t in tensors[1:]:
            out.add_(t)
        return out

    # ---------------------------------------------------------------- MI355X extensions
    def fused_compress(self, tensor: torch.Tensor, name: str, memory: Memory):
        """compensate + compress + update in one native pass; ``None`` = not supported."""
        return None

    def wire_counts(self, tensors: Sequence[torch.Tensor]):
        """The variable-length parts of a fixed-capacity payload with in-band counts
        (ops/cappayload.py): per payload tensor None (fixed) or ``(count_tensor, [esz...])`` --
        its valid bytes are sum_j esz_j * count_tensor[j] (int32 words).  A count-aware
        transport (the xGMI one-shot all-gather) then moves only those bytes.  None (default):
        the whole payload is fixed-size."""
        return None

    def decompress_aggregate(self, per_rank: Sequence[Sequence[torch.Tensor]], ctx: Any,
                             world_size: int) -> torch.Tensor:
        """Decompress every rank's payload, aggregate, and average if ``self.average``.
        Generic version == reference Allgather.send_receive tail (allgather.py:40-45)."""
        dec = [self.decompress(p, ctx) for p in per_rank]
        agg = self.aggregate(dec)
        return agg / world_size if self.average else agg

    def decompress_reduced(self, tensors: Sequence[torch.Tensor], ctx: Any, world_size: int) -> torch.Tensor:
        """Decompress a payload that was SUM-allreduced across ranks (Allreduce communicator).
        Default == reference allreduce.py:9-13: divide each payload by W if averaging, then
        decompress."""
        if self.average:
            tensors = [t.div_(world_size) if t.is_floating_point() else t // world_size for t in tensors]
        return self.decompress(tensors, ctx)


class Communicator(Stateful, ABC):
    """Runs the GRACE pipeline and the collective (reference dist/__init__.py:37-51)."""

    def __init__(self, compressor: Compressor, memory: Memory, world_size: Optional[int] = None,
                 comm=None):
        from .parallel.comm import default_comm

        self.compressor = compressor
        self.memory = memory
        self.profiler = None  # grace_amd.utils.profiler.GraceProfiler (opt-in)
        self._comm_t0 = {}  # id(handles) -> profiler start event of the collective
        self.comm = comm if comm is not None else default_comm()
        self.world_size = int(world_size) if world_size is not None else self.comm.world_size
        if self.world_size != self.comm.world_size:
            raise ValueError(f"world_size={self.world_size} but the process group has {self.comm.world_size} ranks")
        # let compressors that communicate inside compress (PowerSGD) or memories that
        # all-reduce (DGC clipping) use the same explicit comm handle
        for part in (compressor, memory):
            if hasattr(part, "bind_comm"):
                part.bind_comm(self.comm)

    # -------------------------------------------------------------- reference dist API
    def step(self, tensor: torch.Tensor, name: str) -> torch.Tensor:
        handles, ctx = self.send_step(tensor, name)
        return self.receive_step(handles, ctx)

    def send_receive(self, tensors, name, ctx):
        return self.wait_receive(self.async_send(tensors, name), ctx)

    # -------------------------------------------------------------- split-phase API
    def _prof(self):
        from .utils.profiler import NULL

        return self.profiler if self.profiler is not None else NULL

    def compress_step(self, tensor: torch.Tensor, name: str):
        with self._prof().phase("compress", name):
            fused = self.compressor.fused_compress(tensor, name, self.memory)
            if fused is not None:
                return fused
            tensor = self.memory.compensate(tensor, name)
            payload, ctx = self.compressor.compress(tensor, name)
            self.memory.update(tensor, name, self.compressor, payload, ctx)
            return payload, ctx

    def send_step(self, tensor: torch.Tensor, name: str):
        payload, ctx = self.compress_step(tensor, name)
        prof = self._prof()
        prof.add_bytes(sum(t.numel() * t.element_size() for t in payload))
        t0 = prof.start()
        handles = self.async_send(payload, name)
        if t0 is not None:  # comm = the collective on the issuing stream: exact for in-stream
            # collectives (LocalComm, the inline native RCCL runtime); for collectives forked to
            # another stream it is the issue cost (their completion is in the decompress wait)
            prof.stop("comm", t0)
        return handles, ctx

    def receive_step(self, handles, ctx):
        with self._prof().phase("decompress", ""):
            return self.wait_receive(handles, ctx)

    def wait_comm(self, handles) -> None:
        """Make the current stream wait for the collective(s) of ``handles`` (idempotent; the
        decode in ``wait_receive`` then finds them complete).  Default: nothing separable."""

    @abstractmethod
    def async_send(self, tensors: Sequence[torch.Tensor], name: str):
        """Launch the collective(s); returns an opaque handle."""

    @abstractmethod
    def wait_receive(self, handles, ctx) -> torch.Tensor:
        """Wait for the collective(s) and return the aggregated tensor."""

    # -------------------------------------------------------------- checkpointing
    def state_dict(self):
        return {"compressor": self.compressor.state_dict(), "memory": self.memory.state_dict()}

    def load_state_dict(self, state):
        self.compressor.load_state_dict(state.get("compressor", {}))
        self.memory.load_state_dict(state.get("memory", {}))
