"""Weight gradients on a side stream: the backward critical path is dgrad -> BN backward ->
dgrad -> ...; every weight gradient (wgrad) hangs off it and is consumed only by the GRACE
exchange / optimizer after backward.

In a ResNet-50 backward the fused-BN passes are latency bound (a few MB per launch, a serial
fold tail) and the wgrad GEMMs are MFMA bound, yet on one stream every kernel waits for the
one before it.  Here each conv's backward issues its dgrad on the current (critical) stream and
its wgrad on a per-device side stream that first waits for the conv's output gradient: the
wgrad of layer L runs while the BN backward and dgrad of layer L-1 run, so latency-bound
launches share the chip with MFMA work instead of leaving it idle.  In a whole-step HIP graph
the fork becomes a parallel branch of the graph (no host involvement at replay).

Who may fork: only parameters whose gradient consumer is known to join (``mark_joinable``: the
GRACE engine tags its own parameters).  Plain DDP, post-accumulate-grad hooks or user code that
reads ``p.grad`` mid-backward would read a gradient the side stream may still be writing, so
every untagged parameter computes its weight gradient in line.

Joins: (1) the GRACE engine's bucket launch (parallel/engine.py ``_launch`` / ``synchronize``)
makes its consuming stream wait for every wgrad issued so far; (2) a final-callback of every
backward that forked joins the side stream into the caller's current stream, so a user reading
``p.grad`` after ``loss.backward()`` sees finished gradients.  Tensors crossing streams are
tagged with ``record_stream`` so the caching allocator never recycles them early (inside a
capture their reuse is deferred to the end of the capture).

The gradient tensors are handed to autograd without extra references, so AccumulateGrad steals
them (no copy kernel on the critical stream before the join).

``GRACE_WGRAD_STREAM=0`` runs every wgrad in line (A/B knob).  The horovod-style ordering the
reference relies on -- gradients exchanged as they become ready, after their producing kernels
(/root/reference/patch_files/horovod/torch/__init__.py:107-141) -- is kept by join (1).
"""
from __future__ import annotations

import os
import threading
from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

_ENABLED = os.environ.get("GRACE_WGRAD_STREAM", "1") == "1"
# debug / race detector: a spin of this many GPU cycles at every fork on the side stream, so any
# consumer that reads a side-stream weight gradient without joining reads a stale one
_SIDE_DELAY = int(os.environ.get("GRACE_WGRAD_SIDE_DELAY", "0"))
_streams: Dict[int, "torch.cuda.Stream"] = {}
_pending: Dict[int, bool] = {}  # device -> side work issued since the last join
_lock = threading.Lock()


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def enabled() -> bool:
    return _ENABLED


def side_cu_mask(spec: str, n_cu: int):
    """CU-mask words for GRACE_SIDE_CUS: "k/m" keeps k of every m consecutive CUs (spread over
    every XCD / shader engine), e.g. "3/4" = 192 of 256 CUs; "" or "all" = no mask."""
    spec = (spec or "").strip()
    if spec in ("", "all"):
        return []
    k, m = (int(v) for v in spec.split("/"))
    if not (0 < k <= m):
        raise ValueError(f"GRACE_SIDE_CUS={spec!r}: need 0 < k <= m")
    words = [0] * ((n_cu + 31) // 32)
    for cu in range(n_cu):
        if cu % m < k:
            words[cu // 32] |= 1 << (cu % 32)
    return words


_dedicated = {}


def dedicated_stream(idx: int, priority: int = 0, role: str = "side") -> "torch.cuda.Stream":
    """A HIP stream of its own (hipStreamCreateWithPriority), one per (device, priority), kept for
    the process.  torch.cuda.Stream() hands out streams round-robin from a pool of 32 per
    priority, so two of them can be the SAME stream: a split capture's main stream once came back
    as the cached side stream (its second concurrent capture then began on a stream already
    capturing), and a side stream that aliases the caller's serialises the two graphs.  One
    stream per (device, priority, role)."""
    key = (idx, priority, role)
    s = _dedicated.get(key)
    if s is None:
        with _lock:
            s = _dedicated.get(key)
            if s is None:
                from . import _native

                if _native.available():
                    s = torch.cuda.ExternalStream(_native.lib().create_stream(idx, priority),
                                                  device=torch.device("cuda", idx))
                else:
                    with torch.cuda.device(idx):
                        s = torch.cuda.Stream(priority=priority)
                _dedicated[key] = s
    return s


def _side(device: torch.device) -> "torch.cuda.Stream":
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.get(idx)
    if s is None:
        mask = side_cu_mask(os.environ.get("GRACE_SIDE_CUS", ""),
                            torch.cuda.get_device_properties(idx).multi_processor_count)
        with _lock:
            s = _streams.get(idx)
            if s is None and mask:  # the side GEMMs may not take the CUs the critical chain needs
                from . import _native

                ptr = _native.lib().create_stream(idx, 0, mask)
                s = _streams[idx] = torch.cuda.ExternalStream(ptr, device=torch.device("cuda", idx))
        if s is None:
            # a stream of its own, never one of torch's pooled streams (see dedicated_stream); a
            # high-priority side stream measured 20 ms/step (r3_graph_fork_knobs)
            s = _streams[idx] = dedicated_stream(idx, 0, "side")
    return s


def _final_join():
    if _split:  # a split capture joins at its split point (the engine's launch), not here
        return
    join()


# ---------------------------------------------------------------- split-stream capture
# GraphedStep(split=True) (parallel/graph.py) captures a step as TWO linear graphs instead of one
# forked graph: the critical stream's work (A) and this module's side stream (B), joined by
# external event nodes (csrc/runtime/graph_split.cpp ExtEvent).  While such a capture is active
# on a device, ``fork`` records an ExtEvent on the critical stream and the side stream waits on it
# (one event per fork point: the graphs keep referring to them), the end-of-backward join is
# skipped, and the FIRST ``join`` on the critical stream -- the GRACE engine's bucket launch,
# deferred to ``synchronize`` while a split capture runs -- ends both captures and starts the
# critical stream's second graph (A2: the exchange + optimizer).  Replay runs A on the critical
# stream, B on the side stream, joins them eagerly and replays A2.  Each graph is a single
# chain, which the HIP runtime launches as one packet batch; a forked graph is launched node by
# node.
class SplitCapture:
    """State of one split capture on one device.  ``sync`` picks how graph B waits for graph A at
    a fork point: "flags" (default) = one-thread kernels -- A publishes its generation into a flag
    word, B spins on it (bounded) -- so both graphs are pure kernel chains; "events" = external
    event record / wait nodes (measured: every event-record node on the critical stream costs a
    ~60 us gap, profiles/r6_graph_split.txt)."""

    MAX_FORKS = 1024

    def __init__(self, device_idx: int, main: "torch.cuda.Stream", side: "torch.cuda.Stream", on_split,
                 sync: str = "flags", spin_limit: int = 1 << 24):
        from . import _native

        if sync not in ("flags", "events"):
            raise ValueError(f"sync must be 'flags' or 'events', not {sync!r}")
        self.idx = device_idx
        self.main = main
        self.side = side
        self.on_split = on_split   # ends the A / B captures, begins A2 on ``main``
        self.sync = sync
        # one flag per 2 fork points: 2601 -> 2684-2689 img/s (every 3: 2680, 4: 2652, 8: 2662, 13: 2627,
        # 27: 2565; DDP 2558 -> 2649 at 2), profiles/r6_graph_split.txt
        self.every = max(1, int(os.environ.get("GRACE_SPLIT_SYNC_EVERY", "2")))
        self.spin_limit = int(spin_limit)
        self.events = []           # fork-point tokens (ExtEvents stay alive as long as the graphs)
        self.split_done = False
        self._lib = _native.lib()
        dev = torch.device("cuda", device_idx)
        self.flags = torch.zeros(self.MAX_FORKS, dtype=torch.int64, device=dev)
        # the side stream's PROGRESS: bflags[g] = B's generation once every weight gradient of
        # fork group g is done -- the post-join graph A2 waits on these per bucket instead of on
        # the whole side graph (``wait_params``), so one bucket's exchange overlaps the last
        # group's weight gradients
        self.bflags = torch.zeros(self.MAX_FORKS, dtype=torch.int64, device=dev)
        self.group_of = {}     # id(param) -> fork group of its weight gradient
        self.waited = -1       # highest progress group A2 already waited for
        self.gen = torch.zeros(2, dtype=torch.int64, device=dev)  # [A's generation, B's generation]
        # GRACE_SPLIT_TRACE=1: per fork point, the device clock when A signalled it and when B's
        # wait returned (``timeline()``): the two graphs' overlap without a profiler
        self.times = torch.zeros(2 * self.MAX_FORKS, dtype=torch.int64, device=dev) \
            if os.environ.get("GRACE_SPLIT_TRACE", "0") == "1" else None

    def begin_main(self) -> None:
        """First node of graph A (and of every eager use): A's generation += 1."""
        if self.sync == "flags":
            self._lib.xs_bump(self.gen[0:1], self.main.cuda_stream)

    def begin_side(self) -> None:
        """First node of graph B: B's generation += 1 (B waits for flags reaching it)."""
        if self.sync == "flags":
            self._lib.xs_bump(self.gen[1:2], self.side.cuda_stream)

    def signal(self, stream: "torch.cuda.Stream"):
        """Fork point on the critical stream: side work issued after ``wait(token)`` may start.
        Flag sync with ``every = k > 1``: one flag per group of k fork points, published at the
        group's LAST fork (every dy of the group is ready by then); the side stream waits once,
        at the group's first fork -- k times fewer kernels on the critical chain, the side work
        starting up to k - 1 layers later."""
        i = len(self.events)
        if self.sync == "events":
            tok = self._lib.ExtEvent(self.idx)
            tok.record(stream.cuda_stream)
        else:
            if i >= self.MAX_FORKS:
                raise RuntimeError(f"split capture: more than {self.MAX_FORKS} fork points")
            tok = i
            if i % self.every == self.every - 1:
                self._lib.xs_signal(self.flags, i // self.every, self.gen[0:1], stream.cuda_stream, self.times)
        self.events.append(tok)
        return tok

    def wait(self, tok, stream: "torch.cuda.Stream", param=None) -> None:
        if param is not None and self.sync == "flags":
            self.group_of[id(param)] = tok // self.every
        if self.sync == "events":
            tok.wait(stream.cuda_stream)
        elif tok % self.every == 0:  # later forks of the group: already behind that wait
            if tok:  # everything of the previous group is enqueued on B: its progress flag
                self._lib.xs_signal(self.bflags, tok // self.every - 1, self.gen[1:2], stream.cuda_stream, None)
            self._lib.xs_wait(self.flags, tok // self.every, self.gen[1:2], self.spin_limit, stream.cuda_stream,
                              self.times)

    def close_progress(self) -> None:
        """Before the side graph ends: the last group's progress flag."""
        n = len(self.events)
        if self.sync == "flags" and n:
            self._lib.xs_signal(self.bflags, (n - 1) // self.every, self.gen[1:2], self.side.cuda_stream, None)

    def n_groups(self) -> int:
        return -(-len(self.events) // self.every) if self.sync == "flags" else len(self.events)

    def wait_params(self, params, stream: "torch.cuda.Stream") -> None:
        """In A2: wait until the side stream finished the weight gradients of ``params`` (all
        groups up to the latest one holding any of them; ``params=None``: all of them)."""
        if self.sync != "flags":
            raise RuntimeError("per-bucket waits need the flag sync")
        if params is None:
            g = self.n_groups() - 1
        else:
            gs = [self.group_of[id(p)] for p in params if id(p) in self.group_of]
            g = max(gs) if gs else -1
        if g > self.waited:  # progress is monotone: one wait covers every earlier group
            self._lib.xs_wait(self.bflags, g, self.gen[0:1], self.spin_limit, stream.cuda_stream, None)
            self.waited = g

    def close_group(self) -> None:
        """Before the critical stream's graph ends: publish a partly filled last group."""
        n = len(self.events)
        if self.sync == "flags" and n % self.every:
            self._lib.xs_signal(self.flags, n // self.every, self.gen[0:1], self.main.cuda_stream, self.times)

    def timeline(self):
        """[(fork, A signalled (us, from fork 0), B's wait returned (us), B lag (us))] of the last
        replay (GRACE_SPLIT_TRACE=1; the device clock runs at 100 MHz)."""
        if self.times is None:
            return []
        n = -(-len(self.events) // self.every)
        t = self.times[: 2 * n].view(n, 2).cpu().tolist()
        base = t[0][0]
        rows = [(i, (a - base) / 100.0, (b - base) / 100.0, (b - a) / 100.0) for i, (a, b) in enumerate(t)]
        # markers (when recorded): the side graph's end and the post-join graph's start
        m = self.times[2 * (self.MAX_FORKS - 2):].view(2, 2)[:, 0].cpu().tolist()
        if m[0] and m[1]:
            rows.append(("B end / A2 start", (m[0] - base) / 100.0, (m[1] - base) / 100.0, (m[1] - m[0]) / 100.0))
        return rows

    def mark(self, which: str) -> None:
        """GRACE_SPLIT_TRACE: device-clock marker at the side graph's end ("b_end", on the side
        stream) or the post-join graph's start ("a2_start", on the critical stream)."""
        if self.times is None or self.sync != "flags":
            return
        idx, st = (self.MAX_FORKS - 2, self.side) if which == "b_end" else (self.MAX_FORKS - 1, self.main)
        self._lib.xs_signal(self.flags, idx, self.gen[0:1], st.cuda_stream, self.times)

    def split(self):
        if not self.split_done:
            self.split_done = True
            self.close_group()
            if self.sync == "flags":
                with torch.cuda.stream(self.side):
                    self.close_progress()
            self.on_split()


_split: Dict[int, SplitCapture] = {}


def begin_split(sc: SplitCapture) -> None:
    _split[sc.idx] = sc


def end_split(idx: int) -> Optional[SplitCapture]:
    _pending[idx] = False
    return _split.pop(idx, None)


def split_active(device) -> bool:
    """A split capture runs on ``device`` and has not reached its join yet."""
    if not _split:
        return False
    idx = device.index if isinstance(device, torch.device) else device
    sc = _split.get(idx)
    return sc is not None and not sc.split_done


def mark_joinable(params, on: bool = True) -> None:
    """Declare that the consumer of these parameters' gradients joins the side stream (``join``)
    before it reads them: their weight gradients may then run on the side stream.  The GRACE
    engine marks its own parameters; everything else computes weight gradients in line."""
    for p in params:
        if on:
            p._grace_wgrad_join = True
        elif hasattr(p, "_grace_wgrad_join"):
            del p._grace_wgrad_join


def joinable(param: torch.Tensor) -> bool:
    return bool(getattr(param, "_grace_wgrad_join", False))


# GRACE_WGRAD_FORK: which weight gradients may leave the critical stream (A/B of where the side
# stream's gain comes from; every fork point costs the critical stream a dependency marker in a
# split capture).  Comma list of selectors, a conv forks when one matches: "all" (default),
# "k3" / "k1" (kernel size), "hN" (the output gradient's height, e.g. h56 = ResNet stage 1).
_FORK_SEL = tuple(v.strip() for v in os.environ.get("GRACE_WGRAD_FORK", "all").split(",") if v.strip())


def fork_selected(dy: torch.Tensor, w: torch.Tensor) -> bool:
    if "all" in _FORK_SEL:
        return True
    for sel in _FORK_SEL:
        if sel in ("k3", "k1") and w.dim() == 4 and w.shape[-1] == int(sel[1]):
            return True
        if sel.startswith("h") and dy.dim() == 4 and sel[1:].isdigit() and dy.shape[2] == int(sel[1:]):
            return True
    return False


class fork:
    """``f = fork(t)`` marks the current stream's position NOW (before the caller issues its
    critical-path kernels); ``with f as go:`` then runs the body on the side stream of ``t``'s
    device, ordered after that mark only.  ``go`` is False (body runs in line, on the current
    stream) for CPU tensors or when disabled."""

    def __init__(self, t: torch.Tensor, param: Optional[torch.Tensor] = None):
        self.t = t
        self.param = param
        self.ctx = None
        self.main = None
        self.ev = None
        # Only a parameter whose gradient consumer is KNOWN to join the side stream before
        # reading it may fork (``joinable``): the GRACE engine's parameters (it joins at every
        # bucket launch) and explicitly tagged ones.  Any other consumer -- plain DDP, a
        # post-accumulate-grad hook, a user reading p.grad mid-backward -- reads the gradient on
        # the current stream while the side stream may still be writing it, so those stay in
        # line.  A parameter that already holds a .grad gets the new one ADDED by AccumulateGrad
        # on the current stream right after this backward returns: in line as well.  So does a
        # parameter whose gradient a DistributedDataParallel reducer consumes (parallel/ddp_hook.py
        # clears the tag: the reducer reads it from its AccumulateGrad hook, mid-backward).
        self.sc = None
        if (_ENABLED and t.is_cuda and param is not None and param.grad is None and joinable(param)
                and fork_selected(t, param) and (not must_alias(param) or grad_target(param) is not None)):
            # (a gradient its consumer reads mid-backward from a bucket view -- the deferred DDP
            # hook's reducer -- may leave the critical stream only once that view is known and
            # stable: the side stream then writes INTO it and the reducer reads nothing)
            sc = _split.get(t.device.index)
            if sc is not None and sc.split_done:
                return  # after the split's join (A2): nothing may fork any more, stay in line
            self.main = torch.cuda.current_stream(t.device)
            if sc is not None:  # split capture: a fork point graph B waits on (flag word / event node)
                if self.main.cuda_stream != sc.main.cuda_stream:
                    return
                self.sc = sc
                self.ev = sc.signal(self.main)
            else:
                self.ev = torch.cuda.Event()
                self.ev.record(self.main)

    def __enter__(self) -> bool:
        if self.ev is None:
            return False
        t = self.t
        side = _side(t.device)
        if self.sc is not None:
            self.sc.wait(self.ev, side, self.param)
        else:
            side.wait_event(self.ev)
        self.ctx = torch.cuda.stream(side)
        self.ctx.__enter__()
        if _SIDE_DELAY:  # race detector: the side stream lags far behind the critical stream
            torch.cuda._sleep(_SIDE_DELAY)
        idx = t.device.index
        if self.sc is not None:  # the split's join (``join`` on the critical stream) ends it
            _pending[idx] = True
        elif not _pending.get(idx):
            _pending[idx] = True
            # one final callback per backward pass: join before backward() returns
            try:
                torch.autograd.Variable._execution_engine.queue_callback(_final_join)
            except RuntimeError:  # not inside a backward pass
                pass
        return True

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
        return False


# ---------------------------------------------------------------- gradients straight into the bucket
# The GRACE engine (parallel/engine.py) marks each dense parameter with the bucket view its
# gradient belongs in (``_grace_grad_view``).  When the parameter has no .grad yet (the
# zero_grad(set_to_none=True) step), a weight-gradient producer may write the gradient into that
# view directly -- on the side stream, off the critical path -- and return a fresh alias of it:
# AccumulateGrad steals the alias, the engine sees a gradient that already lives in its bucket,
# and the per-bucket gather launch (a full read + write of every gradient on the critical path
# after the join) has nothing left to copy.  GRACE_WGRAD_DIRECT=0 disables it.
_DIRECT = os.environ.get("GRACE_WGRAD_DIRECT", "1") == "1"


def grad_target(weight: torch.Tensor) -> Optional[torch.Tensor]:
    """The engine's bucket view for ``weight``'s gradient when backward may write it in place."""
    if not _DIRECT:
        return None
    v = getattr(weight, "_grace_grad_view", None)
    if v is None or weight.grad is not None or v.dtype != weight.dtype or v.device != weight.device:
        return None
    if must_alias(weight) and not getattr(weight, "_grace_view_stable", False):
        # a DDP bucket view seen on only one hook call may be replaced by DDP's bucket rebuild
        # (after the first iteration): the reducer would then find no alias and copy mid-backward
        return None
    return v


def must_alias(weight: torch.Tensor) -> bool:
    """The gradient's consumer reads it mid-backward from the parameter's bucket view -- a DDP
    reducer with the GRACE comm hook deferred (parallel/ddp_hook.py ``defer``): a side-stream
    gradient must then be written INTO that view (the reducer finds an alias and copies
    nothing), whatever produced it, library kernels included."""
    return bool(getattr(weight, "_grace_alias_grad", False))


def into_target(dw: torch.Tensor, tgt: Optional[torch.Tensor]) -> torch.Tensor:
    """dw written into tgt (if given; a no-op when dw already is tgt's memory), returned as a FRESH
    alias of tgt (no other reference: AccumulateGrad steals it instead of cloning)."""
    if tgt is None:
        return dw
    if dw.data_ptr() != tgt.data_ptr():
        tgt.copy_(dw.view_as(tgt) if dw.shape == tgt.shape else dw.reshape(tgt.shape))
    return tgt.view_as(tgt)


def tag(t: Optional[torch.Tensor], stream: "torch.cuda.Stream") -> None:
    """The caching allocator must not recycle ``t`` before ``stream``'s work on it ran."""
    if t is not None and t.is_cuda:
        t.record_stream(stream)


def join(stream: Optional["torch.cuda.Stream"] = None, device=None, params=None) -> None:
    """Make ``stream`` (default: the current stream) wait for every side-stream wgrad issued so
    far.  In a split capture the first join on the capture stream ends graphs A and B; from
    then on (graph A2) a join is a device-side wait for the side stream's progress -- of the
    weight gradients of ``params`` only, when given (the engine's per-bucket launch)."""
    if _split:
        idx = (stream.device.index if stream is not None else
               (torch.device(device).index if device is not None and not isinstance(device, int) else
                device if device is not None else torch.cuda.current_device()))
        sc = _split.get(idx)
        if sc is not None and (sc.split_done or _pending.get(idx)):
            cur = stream if stream is not None else torch.cuda.current_stream(idx)
            if cur.cuda_stream != sc.main.cuda_stream:
                raise RuntimeError("split capture: side-stream weight gradients must be joined on the capture "
                                   "stream (the engine's bucket launch; no overlap stream, no DDP reducer)")
            if not sc.split_done:
                sc.split()  # ends graphs A and B, A2 captures from here
                _pending[idx] = False
            if sc.events and sc.sync == "flags":
                sc.wait_params(params, cur)
            return
    if not _pending:
        return
    if stream is not None:
        devs = [stream.device.index]
    elif device is not None:
        devs = [torch.device(device).index if not isinstance(device, int) else device]
    else:
        devs = [torch.cuda.current_device()]
    for idx in devs:
        if _pending.get(idx):
            tgt = stream if stream is not None else torch.cuda.current_stream(idx)
            tgt.wait_stream(_streams[idx])
            _pending[idx] = False


# ---------------------------------------------------------------- dgrad as a forward convolution
# A stride-1 convolution's data gradient is itself a stride-1 convolution of dy with the
# spatially flipped, in/out-transposed filter (padding k-1-p), so MIOpen's forward solvers are
# an alternative to its backward-data solvers (which zero-fill their output first,
# SubTensorOpWithScalar1d).  The per-shape autotune below times both forms on the device (the
# flipped filter's two small transform kernels charged to the forward form) and keeps the
# faster one; decisions are taken in eager steps only.  Measured on the fp32 ResNet-50 b32 3x3
# layers (profiles/r3_wgrad_side_stream_ab.txt) the backward-data solver wins every shape
# (80-83 us vs 93-110 us per call), so the autotune is opt-in (GRACE_DGRAD_AUTO=1).
_DG_CHOICE = {}
_DG_TIMES = {}
_DG_AUTO = os.environ.get("GRACE_DGRAD_AUTO", "0") == "1"


def dgrad_table():
    """[(key, chosen, {form: ms})] of the autotuned data-gradient forms."""
    return [(k, v, dict(_DG_TIMES.get(k, {}))) for k, v in sorted(_DG_CHOICE.items())]


def _flipped(w):
    return w.permute(1, 0, 2, 3).flip(2, 3).contiguous(memory_format=torch.channels_last)


def _dgrad(dy, x, w, stride, padding, dilation, groups):
    cb = torch.ops.aten.convolution_backward
    kh, kw = w.shape[2], w.shape[3]
    eligible = (_DG_AUTO and dy.is_cuda and groups == 1 and list(stride) == [1, 1] and list(dilation) == [1, 1]
                and (kh > 1 or kw > 1) and padding[0] <= kh - 1 and padding[1] <= kw - 1
                and x.is_contiguous(memory_format=torch.channels_last))

    def bwd():
        return cb(dy, x, w, None, stride, padding, dilation, False, [0, 0], groups, [True, False, False])[0]

    if not eligible:
        return bwd()
    pad = [kh - 1 - padding[0], kw - 1 - padding[1]]

    def fwd():
        return F.conv2d(dy, _flipped(w), None, 1, pad)

    key = (tuple(x.shape), tuple(w.shape), tuple(padding), x.dtype)
    c = _DG_CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            return bwd()
        times = {}
        for name, fn in (("bwd", bwd), ("fwd_flipped", fwd)):
            for _ in range(2):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                fn()
            e.record()
            e.synchronize()
            times[name] = s.elapsed_time(e) / 5
        c = min(times, key=times.get)
        _DG_CHOICE[key] = c
        _DG_TIMES[key] = times
    return fwd() if c == "fwd_flipped" else bwd()


# ---------------------------------------------------------------- convolution with a forked wgrad
class _ConvSplitFn(torch.autograd.Function):
    """conv2d (no bias) whose backward issues dgrad in line and wgrad on the side stream
    (``aten.convolution_backward`` once per direction: MIOpen runs them as two solvers anyway)."""

    @staticmethod
    def forward(ctx, x, weight, stride, padding, dilation, groups):
        ctx.save_for_backward(x, weight)
        ctx.conf = (stride, padding, dilation, groups)
        return F.conv2d(x, weight, None, stride, padding, dilation, groups)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, padding, dilation, groups = ctx.conf
        cb = torch.ops.aten.convolution_backward
        dx = dw = None
        f = fork(dy, w) if ctx.needs_input_grad[1] else None

        def wg():
            # MIOpen returns its own gradient tensor: writing it into the bucket view would be one
            # more copy kernel per conv at the END of the side stream (the step's critical tail
            # once the dgrad chain is done); the engine's single gather launch copies these
            with f as side:
                d = cb(dy, x, w, None, stride, padding, dilation, False, [0, 0], groups, [False, True, False])[1]
                if must_alias(w):
                    d = into_target(d, grad_target(w))
                if side:
                    s = torch.cuda.current_stream(dy.device)
                    tag(dy, s)
                    tag(x, s)
                    tag(d, f.main)
            return d

        if ctx.needs_input_grad[0]:
            dx = _dgrad(dy, x, w, stride, padding, dilation, groups)
        if f is not None:  # issued after the in-line dgrad (before it measured slower, r3_graph_fork_knobs)
            dw = wg()
        return dx, dw, None, None, None, None


def _as2(v):
    return list(v) if isinstance(v, (tuple, list)) else [v, v]


class Conv2dSplitGrad(nn.Conv2d):
    """``nn.Conv2d`` (same parameters / state_dict) whose weight gradient runs on the side stream
    on GPU; bias / string padding / non-zero padding modes / CPU fall back to ``nn.Conv2d``."""

    def forward(self, x):
        if (self.kernel_size == (3, 3) or self.stride != (1, 1)) and x.is_cuda:
            from . import conv as _conv  # (conv imports this module)

            if _conv.conv3x3_ok(x, self):  # implicit GEMM on the f32 MFMA kernel, autotuned vs MIOpen
                return _conv._Conv3x3Fn.apply(x, self.weight, self.stride[0])
        if (_ENABLED and x.is_cuda and self.bias is None and self.padding_mode == "zeros"
                and not isinstance(self.padding, str) and torch.is_grad_enabled() and self.weight.requires_grad):
            w = self.weight
            if torch.is_autocast_enabled():
                # autocast: only when the parameter already IS in the autocast dtype (bf16 working
                # copies, parallel/precision.py) -- a per-step cast of an fp32 weight would put its
                # backward copy on the compute stream, reading the side stream's gradient early
                if w.dtype != torch.get_autocast_dtype("cuda"):
                    return super().forward(x)
                if x.dtype != w.dtype and x.is_floating_point():
                    x = x.to(w.dtype)
            if x.dtype == w.dtype:
                return _ConvSplitFn.apply(x, w, _as2(self.stride), _as2(self.padding), _as2(self.dilation),
                                          self.groups)
        return super().forward(x)
