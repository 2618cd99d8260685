"""Process-group bootstrap, timeouts and a comm watchdog (failure detection).

The reference's only failure handling is ``init_process_group(timeout=20 s)``
(/root/reference/examples/dist/CIFAR10-dawndist/core.py:225-226).  Here:

* ``init_distributed`` reads torchrun's env (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*),
  pins the GPU, picks RCCL ("nccl") on GPUs and gloo on CPU, enables RCCL async error
  handling and applies a finite collective timeout;
* ``Watchdog`` tracks in-flight GRACE collectives and raises (or aborts the native RCCL
  communicator) in the training thread when one exceeds its deadline, instead of hanging
  forever when a peer dies.
"""
from __future__ import annotations

import datetime
import os
import threading
import time
from typing import Optional

import torch
import torch.distributed as dist


def init_distributed(backend: Optional[str] = None, timeout_s: float = 300.0):
    """Initialise torch.distributed from the torchrun environment; returns (rank, world, device)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        backend = backend or "nccl"  # = RCCL on ROCm
    else:
        device = torch.device("cpu")
        backend = backend or "gloo"
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": device} if device.type == "cuda" else {}
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world, device


class Watchdog:
    """Deadline monitor for async collectives.

    ``track(work, what)`` registers a handle; a daemon thread polls ``work.is_completed()`` and
    records a failure when the deadline passes.  ``check()`` (call it once per step, e.g. from
    the optimizer) raises ``TimeoutError`` in the training thread; with ``abort=comm`` the
    native RCCL communicator is aborted so the stuck kernels are torn down (from the watchdog
    thread: a training thread blocked on the hung collective cannot do it itself; the native
    runtime serialises abort against in-flight issue calls, csrc/comm/rccl_comm.cpp).
    ``track_stream(what)`` records an event on the current stream -- the engine calls it after
    each step's collectives so a dead peer becomes a TimeoutError instead of a silent hang.
    """

    def __init__(self, timeout_s: float = 120.0, poll_s: float = 0.5, abort=None):
        self.timeout_s = timeout_s
        self.poll_s = poll_s
        self.abort = abort
        self._items = []
        self._lock = threading.Lock()
        self._failure: Optional[str] = None
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, daemon=True, name="grace-watchdog")
        self._thread.start()

    def track(self, work, what: str = "collective"):
        if work is None:
            return
        with self._lock:
            self._items.append((time.monotonic() + self.timeout_s, work, what))

    def track_stream(self, what: str = "step collectives"):
        """Track completion of everything queued so far on the current stream."""
        if not torch.cuda.is_available():
            return
        ev = torch.cuda.Event()
        ev.record()

        class _Ev:
            def is_completed(self_inner):
                return ev.query()

        self.track(_Ev(), what)

    def _run(self):
        while not self._stop.wait(self.poll_s):
            now = time.monotonic()
            with self._lock:
                keep = []
                for deadline, work, what in self._items:
                    try:
                        done = work.is_completed()
                    except Exception as e:  # the backend already reported an error
                        self._failure = f"{what}: {e!r}"
                        continue
                    if done:
                        continue
                    if now > deadline:
                        self._failure = f"{what} did not complete within {self.timeout_s:.0f}s"
                        if self.abort is not None:
                            try:
                                self.abort.abort()
                            except Exception:
                                pass
                        continue
                    keep.append((deadline, work, what))
                self._items = keep

    def check(self):
        if self._failure:
            raise TimeoutError(f"grace watchdog: {self._failure}")

    def close(self):
        self._stop.set()
        self._thread.join(timeout=2)
