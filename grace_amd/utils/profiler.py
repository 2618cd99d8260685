"""Opt-in GRACE profiler: per-phase GPU time without host syncs on the hot path.

The reference only has ad-hoc ``torch.cuda.synchronize(); time.time(); print`` inside the
Horovod QSGD compressor (/root/reference/grace_dl/torch/compressor/qsgd.py:14-15, 33-34) and
commented compute/communication prints in the benchmark (pytorch_synthetic_benchmark.py:
166-167).  Here every phase of the pipeline (compress = compensate+compress+update, comm =
collective issue->completion as seen by the consuming stream, decompress = decompress +
aggregate) is bracketed by a pair of
``torch.cuda.Event`` s recorded on the stream that runs it, plus a roctx range (visible in
``rocprofv3 --marker-trace``).  Events are resolved only when ``report()`` is called.

    prof = GraceProfiler(); grc.profiler = prof
    ... train ...
    print(prof.report())   # {"compress": ms/step, "comm": ..., "decompress": ..., "bytes": ...}
"""
from __future__ import annotations

import contextlib
from collections import defaultdict
from typing import Dict, List, Tuple

import torch


class GraceProfiler:
    def __init__(self, enabled: bool = True, roctx: bool = True):
        self.enabled = enabled
        self.roctx = roctx
        self._pending: List[Tuple[str, torch.cuda.Event, torch.cuda.Event]] = []
        self._totals: Dict[str, float] = defaultdict(float)
        self._counts: Dict[str, int] = defaultdict(int)
        self.bytes_sent = 0
        self.steps = 0

    @contextlib.contextmanager
    def phase(self, name: str, tag: str = ""):
        if not self.enabled or not torch.cuda.is_available():
            yield
            return
        if self.roctx:
            torch.cuda.nvtx.range_push(f"grace.{name}:{tag}")
        start = torch.cuda.Event(enable_timing=True)
        end = torch.cuda.Event(enable_timing=True)
        start.record()
        try:
            yield
        finally:
            end.record()
            if self.roctx:
                torch.cuda.nvtx.range_pop()
            self._pending.append((name, start, end))

    def start(self):
        """Event marking the start of a span that ends in another call (``stop``)."""
        if not self.enabled or not torch.cuda.is_available():
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def stop(self, name: str, start) -> None:
        if start is None:
            return
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        self._pending.append((name, start, end))

    def add_bytes(self, n: int):
        self.bytes_sent += int(n)

    def step(self):
        self.steps += 1

    def _resolve(self):
        for name, s, e in self._pending:
            e.synchronize()
            self._totals[name] += s.elapsed_time(e)
            self._counts[name] += 1
        self._pending.clear()

    def report(self) -> Dict[str, float]:
        self._resolve()
        steps = max(1, self.steps)
        out = {f"{k}_ms_per_step": v / steps for k, v in self._totals.items()}
        out["bytes_per_step"] = self.bytes_sent / steps
        out["steps"] = self.steps
        return out

    def reset(self):
        self._resolve()
        self._totals.clear()
        self._counts.clear()
        self.bytes_sent = 0
        self.steps = 0


class _Null:
    @contextlib.contextmanager
    def phase(self, name, tag=""):
        yield

    def start(self):
        return None

    def stop(self, name, start):
        pass

    def add_bytes(self, n):
        pass


NULL = _Null()
