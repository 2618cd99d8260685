"""Whole-training-step HIP-graph capture (forward + backward + GRACE exchange + optimizer).

An eager ResNet-50 step issues ~1100 kernels; at a few microseconds of host time each the CPU
launch path is as long as the GPU work.  Capturing the step once into a HIP graph and
replaying it removes the Python/dispatcher cost of every op, every backward hook and every
GRACE kernel launch (MI355X_MICROARCH: graph replay ~10-16 us per replay vs ~3.5 us per eager
launch).

Requirements on the step (checked by construction in grace_amd):
* static shapes and static input buffers (copy new data into them before ``replay``);
* no host synchronisation inside the step -- every built-in codec qualifies except Sketch; the
  variable-size ones (Threshold / DGC / Adaq / INCEPTIONN) exchange FIXED-capacity payloads with
  an in-band count (ops/cappayload.py), so no payload size is read back to the host;
* steady state before capture: the warm-up steps allocate residual / momentum state, so the
  captured kernels read and update it in place on every replay;
* per-step randomness must advance on replay: Random-K indices, QSGD/TernGrad/Natural rounding
  and PowerSGD's Q mix a DEVICE step counter into their seeds (compressor/_base.py DeviceSteps,
  bumped by a captured ``add_(1)``), so they are capturable on the native path.  Their torch
  fallbacks seed a host generator, which a replay would freeze: refused unless
  ``allow_static_seeds=True``.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from . import health as _health

_SYNC_EACH = __import__("os").environ.get("GRACE_GRAPH_SYNC_EACH", "0") == "1"

#: stochastic codecs whose native kernels read a device step counter
_DEVICE_STEPPED = ("RandomKCompressor", "QSGDCompressor", "TernGradCompressor", "NaturalCompressor",
                   "PowerSGDCompressor", "DgcCompressor", "AdaqCompressor")
_HOST_SYNC = ()


def graph_safe(grc, allow_static_seeds: bool = False) -> Optional[str]:
    """None if the GRACE pipeline can be captured, else the reason it cannot."""
    name = type(grc.compressor).__name__
    if name in _HOST_SYNC:
        return f"{name} reads payload sizes back to the host"
    if name == "SketchCompressor":
        from ..ops import _native

        # the native multi-rank select + encode (any q <= 65535) is capturable; the sort path is not
        if grc.compressor.quantiles > 65535 or not _native.available():
            return f"{name} with {grc.compressor.quantiles} quantiles sorts the bucket (no native select)"
    if not grc.compressor.tensors_size_are_same:
        return f"{name} has variable-size payloads"
    if name in _DEVICE_STEPPED and not allow_static_seeds:
        from ..ops import _native

        if not _native.available() or not _native.native_on("cuda"):
            return f"{name} without the native extension draws randomness from host-side seeds"
    return None


def _new_graph() -> "torch.cuda.CUDAGraph":
    """GRACE_GRAPH_CENSUS=1 keeps the raw hipGraph_t inspectable after capture (instantiated on
    the first replay instead of at capture end) for the bench's node census."""
    import os

    if os.environ.get("GRACE_GRAPH_CENSUS", "0") == "1":
        return torch.cuda.CUDAGraph(keep_graph=True)
    return torch.cuda.CUDAGraph()


def _is_rccl_backend(name) -> bool:
    """True for any backend string that includes RCCL: "nccl", and the per-device forms such as
    "cpu:gloo,cuda:nccl" (what ``init_process_group()`` without a backend reports on a GPU box)."""
    return "nccl" in str(name).lower()


def _nccl_group_up() -> bool:
    """Whether any RCCL communicator -- whose threads (the ProcessGroupNCCL watchdog, RCCL's proxy)
    make HIP calls while the training thread captures -- is up in this process: the default
    group, ANY subgroup (a step may run on an NCCL subgroup over a gloo default group), or a live
    native RcclComm (csrc/comm/rccl_comm.cpp)."""
    import torch.distributed as dist

    from . import native_comm

    if native_comm.live_count() > 0:
        return True
    if not (dist.is_available() and dist.is_initialized()):
        return False
    try:
        groups = list(dist.distributed_c10d._world.pg_map.keys())
    except Exception:  # noqa: BLE001 -- private registry moved: the default group alone
        groups = []
    for g in [None] + groups:
        try:
            if _is_rccl_backend(dist.get_backend(g)):
                return True
        except Exception:  # noqa: BLE001 -- a group without a backend: no watchdog to race
            continue
    return False


class GraphedStep:
    """``step = GraphedStep(fn)``; ``step()`` replays the captured ``fn``.

    ``fn`` must perform a full training step on static buffers (zero_grad, forward, backward,
    optimizer.step) and return the loss tensor.

    ``capture_error_mode`` is passed to ``torch.cuda.graph``.  With collectives inside the
    step (W > 1) use ``"thread_local"``: RCCL's proxy thread makes HIP calls of its own while
    the training thread captures, and under ``"global"`` mode such a call from ANY thread
    invalidates the capture.  The default (None) picks ``"thread_local"`` whenever a
    ``torch.distributed`` NCCL (RCCL) group is up -- its watchdog thread queries the events of
    work in flight, which is also such a call -- and ``"global"`` otherwise.

    Every replay first checks the process-wide communication health words (a host-mapped read,
    no device sync): a device-side fault of an earlier replay (an xGMI peer wait that timed out;
    FusedSGD skipped that update) raises :class:`~grace_amd.parallel.health.CommFault` here.
    """

    def __init__(self, fn: Callable[[], torch.Tensor], warmup: int = 3, pool=None,
                 capture_error_mode: Optional[str] = None, copies: Optional[int] = None,
                 stream: Optional[torch.cuda.Stream] = None, split: Optional[bool] = None):
        import os

        self.fn = fn
        self._stream_arg = stream
        if capture_error_mode is None:
            capture_error_mode = "thread_local" if _nccl_group_up() else "global"
        # split: capture the critical stream and the weight-gradient side stream as separate
        # linear graphs joined by flag words / event nodes (ops/wgrad.py SplitCapture); the step
        # must join the side stream only on the capture stream after backward: the GRACE engine
        # without overlap, or DDP with the deferred comm hook (GraceHookState(defer=True))
        if split is None:
            split = os.environ.get("GRACE_GRAPH_SPLIT", "0") == "1"
        self.split = bool(split)
        # ``stream``: warm up, capture and replay on this stream.  Needed when long-lived autograd
        # nodes were created under it -- DDP's reducer keeps the parameters' AccumulateGrad nodes,
        # which run on the stream current at DDP's construction; a capture on any other stream
        # would see them on a non-capturing stream
        side = stream if stream is not None else torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        # copies > 1: the step is captured that many times into one memory pool and the copies
        # are replayed round-robin (stream-ordered, so they may share every buffer).  A forked
        # graph (parallel branches) is launched node by node by the HIP runtime, and a graph
        # cannot be re-submitted while its previous launch still runs; alternating copies lets
        # the host submit step N+1 while step N executes.
        self.g_side = self.g_a2 = None
        self._hp = None  # private high-priority replay stream (split, normal-priority callers)
        if self.split:
            self._capture_split(fn, pool, capture_error_mode)
            return
        copies = int(os.environ.get("GRACE_GRAPH_COPIES", "1")) if copies is None else int(copies)
        # GRACE_GRAPH_PRIORITY=-1: capture and replay on a high-priority stream (the compute
        # stream of the step then outranks the side streams it forks)
        prio = int(os.environ.get("GRACE_GRAPH_PRIORITY", "0"))
        self.stream = stream if stream is not None else (torch.cuda.Stream(priority=prio) if prio else None)
        self.graphs = []
        self.losses = []
        for i in range(max(1, copies)):
            g = _new_graph()
            with torch.cuda.graph(g, pool=pool, stream=self.stream, capture_error_mode=capture_error_mode):
                loss = fn()
            torch.cuda.synchronize()
            if pool is None:
                pool = g.pool()
            self.graphs.append(g)
            # keep the static output, not its autograd graph: the graph would keep the captured
            # AccumulateGrad nodes (bound to the capture stream) alive into later eager
            # backwards on other streams (autograd's stream-mismatch warning and syncs)
            self.losses.append(loss.detach() if isinstance(loss, torch.Tensor) else loss)
        self.graph = self.graphs[0]
        self.loss = self.losses[0]
        self._next = 0

    def _capture_split(self, fn, pool, mode):
        """Graph A (critical stream, until the engine's join), graph B (the wgrad side stream,
        captured at the same time), graph A2 (critical stream, from the join on)."""
        import os

        from ..ops import wgrad as _wg

        dev = torch.cuda.current_device()
        # GRACE_SPLIT_MAIN_PRIO=-1: the critical chain's queue outranks the side queue in the
        # command processor's dispatch arbitration
        # the caller's stream when given (DDP: the reducer's AccumulateGrad nodes run on the stream
        # the model was wrapped under)
        # (a dedicated stream: a pooled torch.cuda.Stream() may be the side stream itself)
        main = self._stream_arg if self._stream_arg is not None else \
            _wg.dedicated_stream(dev, int(os.environ.get("GRACE_SPLIT_MAIN_PRIO", "0")), "split-main")
        side = _wg._side(torch.device("cuda", dev))
        ga, gb, ga2 = _new_graph(), _new_graph(), _new_graph()
        open_ = {"a": False, "b": False, "a2": False}

        def end(g, st, key):
            with torch.cuda.stream(st):
                g.capture_end()
            open_[key] = False

        def on_split():
            sc.mark("b_end")
            end(gb, side, "b")
            end(ga, main, "a")
            # A2 gets its OWN pool: with flag sync it may start while graph B still runs (each
            # bucket waits on the side stream's progress on the device), so it must not reuse
            # blocks graph A freed that B may still read
            with torch.cuda.stream(main):
                ga2.capture_begin(capture_error_mode=mode)
            open_["a2"] = True
            sc.mark("a2_start")

        _health.init()  # the flag waits' timeout raises the process-wide fault words
        sc = _wg.SplitCapture(dev, main, side, on_split, sync=os.environ.get("GRACE_GRAPH_SPLIT_SYNC", "flags"))
        main.wait_stream(torch.cuda.current_stream())
        side.wait_stream(torch.cuda.current_stream())
        torch.cuda.synchronize()
        try:
            with torch.cuda.stream(main):
                ga.capture_begin(pool=pool, capture_error_mode=mode)
            open_["a"] = True
            sc.begin_main()
            with torch.cuda.stream(side):
                gb.capture_begin(capture_error_mode=mode)  # its own pool: A and B replay concurrently
            open_["b"] = True
            sc.begin_side()
            _wg.begin_split(sc)
            try:
                with torch.cuda.stream(main):
                    loss = fn()
            finally:
                _wg.end_split(dev)
            if open_["a2"]:
                end(ga2, main, "a2")
            else:  # no join on the critical stream: A and B only
                sc.close_group()
                end(gb, side, "b")
                end(ga, main, "a")
        except BaseException:
            for key, g, st in (("a2", ga2, main), ("b", gb, side), ("a", ga, main)):
                if open_[key]:
                    try:
                        end(g, st, key)
                    except Exception:  # noqa: BLE001 -- already failing; a live capture aborts at exit
                        pass
            raise
        torch.cuda.synchronize()
        self._sc = sc  # keeps the ExtEvents the graphs' nodes refer to
        self.s_main, self.s_side = main, side
        self.graphs = [ga]
        self.g_side = gb if sc.events else None
        self.g_a2 = ga2 if sc.split_done else None
        self.graph = ga
        self.losses = [loss.detach() if isinstance(loss, torch.Tensor) else loss]
        self.loss = self.losses[0]
        self._next = 0
        self.stream = None

    def _replay_split(self) -> torch.Tensor:
        # a graph is not bound to its capture stream: A and A2 replay on the caller's stream (two
        # cross-stream joins per step instead of four), B on the side stream -- when the caller's
        # stream is high priority.  A and B must sit on different HARDWARE queues, and HIP deals the
        # streams of one priority to a few of them (GPU_MAX_HW_QUEUES): with more streams alive
        # (the native RCCL runtime's) the side stream shared the caller's queue and the two graphs
        # serialised (ResNet-50 2494 vs 2746 img/s, profiles/r6_graph_split.txt).  A normal-priority
        # caller gets its replay moved to a private high-priority stream (bench.py runs the whole
        # step on one, avoiding the two extra joins)
        caller = torch.cuda.current_stream()
        if caller.priority < 0:
            return self._replay_split_on(caller)
        hp = self._hp
        if hp is None:
            from ..ops import wgrad as _wg

            hp = self._hp = _wg.dedicated_stream(caller.device.index, -1, "split-replay")
        hp.wait_stream(caller)
        with torch.cuda.stream(hp):
            loss = self._replay_split_on(hp)
        caller.wait_stream(hp)
        return loss

    def _replay_split_on(self, cur) -> torch.Tensor:
        side = self.s_side
        if self.g_side is not None:
            side.wait_stream(cur)  # after the previous step's A2
        self.graphs[0].replay()
        if self.g_side is not None:
            with torch.cuda.stream(side):
                self.g_side.replay()
            if self._sc.sync != "flags":  # event sync: A2 has no device-side waits on B
                cur.wait_stream(side)
        if self.g_a2 is not None:
            self.g_a2.replay()  # (flag sync: every bucket launch waits on B's progress inside A2)
        if self.g_side is not None:
            cur.wait_stream(side)
        if _SYNC_EACH:
            torch.cuda.synchronize()
        return self.loss

    def __call__(self) -> torch.Tensor:
        _health.check()
        if self.split:
            return self._replay_split()
        i = self._next
        self._next = (i + 1) % len(self.graphs)
        if self.stream is not None:
            cur = torch.cuda.current_stream()
            self.stream.wait_stream(cur)
            with torch.cuda.stream(self.stream):
                self.graphs[i].replay()
            cur.wait_stream(self.stream)
        else:
            self.graphs[i].replay()
        if _SYNC_EACH:  # debug A/B: no replay overlaps the host issue of the next one
            torch.cuda.synchronize()
        self.loss = self.losses[i]
        return self.loss


def graph_compute(model: torch.nn.Module, sample_input: torch.Tensor, engine=None, warmup: int = 3):
    """Capture only the model's forward and backward (``torch.cuda.make_graphed_callables``);
    gradient accumulation, the GRACE exchange and the optimizer stay eager.  Works with any
    communication backend (no collective inside the graph), so it is the multi-GPU-safe graph
    mode; ~1000 eager launches per ResNet-50 step become 2 graph launches.
    ``engine`` (a GraceEngine) is paused during the warm-up/capture backward passes."""
    import contextlib

    ctx = engine.pause() if engine is not None else contextlib.nullcontext()
    with ctx:
        g = torch.cuda.make_graphed_callables(model, (sample_input,), num_warmup_iters=warmup)
    if engine is not None:
        engine.zero_grad()
    return g
