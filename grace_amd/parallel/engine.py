"""Bucketed, overlapped GRACE gradient exchange for one-process-per-GPU data parallelism.

Replaces the reference's per-parameter, serial-after-backward loop
(/root/reference/examples/dist/CIFAR10-dawndist/core.py:203-206) and the Horovod
per-parameter hooks (/root/reference/patch_files/horovod/torch/__init__.py:107-161):

* parameters are grouped into **buckets** (reverse registration order ~ backward order); each
  bucket owns ONE flat fp32 gradient buffer and every ``p.grad`` is a view into it, so the
  compressor sees a whole bucket and its kernels run once per bucket (per-parameter semantics
  are kept through the bucket's :class:`SegmentLayout`);
* a ``post_accumulate_grad`` hook counts ready parameters; when a bucket is complete its
  compress (fused error-feedback kernels) is launched on a dedicated **compress stream** and
  the collective (RCCL over xGMI) is issued asynchronously -- all while the rest of backward
  keeps running on the compute stream;
* ``synchronize()`` makes the compute stream wait for the collectives and runs the one-pass
  decompress/aggregate kernels, writing the averaged gradient back into the bucket buffer.

Bucket sizing for MI355X: xGMI is point-to-point (7 links x ~153 GB/s per GPU); a compressed
bucket of a few MB saturates the links well beyond latency, so the default is few large buckets
(``bucket_cap_mb=64``, whole ResNet-50 = 2 buckets); more buckets = more overlap with backward
but more kernel launches.  288 GB of HBM per GPU makes the extra flat buffers irrelevant.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import health as _health
from ..core import Communicator, register_layout
from ..ops import _native
from ..ops import wgrad as _wgrad
from ..ops.layout import SegmentLayout
from ..ops.randomk import fnv1a64



def _record_stream(obj, stream, _depth=0):
    """Mark every tensor reachable from a handle/ctx as used by ``stream`` so the caching
    allocator does not recycle compress-stream buffers while the compute stream still reads
    them (decompress runs on the compute stream)."""
    if _depth > 6 or obj is None:
        return
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            obj.record_stream(stream)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _record_stream(o, stream, _depth + 1)
    elif isinstance(obj, dict):
        for o in obj.values():
            _record_stream(o, stream, _depth + 1)
    elif hasattr(obj, "__dict__") and not isinstance(obj, type):
        for o in vars(obj).values():
            _record_stream(o, stream, _depth + 1)


class Bucket:
    def __init__(self, name: str, params: List[torch.nn.Parameter], device, dtype=torch.float32):
        self.name = name
        self.params = params
        self.layout = SegmentLayout.from_tensors(params)
        register_layout(name, self.layout)
        self.flat = torch.zeros(self.layout.total, dtype=dtype, device=device)
        self.views = []
        for (_, o, n), p in zip(self.layout.segments(), params):
            seg = self.flat[o:o + n]
            if (not p.is_contiguous() and p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last)):
                # keep the parameter's memory format (channels_last convs): AccumulateGrad then
                # adds in place with no layout-conversion copy; the segment is the gradient's
                # memory image, per-tensor compression is order independent
                v = seg.as_strided(p.shape, p.stride())
            else:
                v = seg.view(p.shape)
            self.views.append(v)
            p.grad = v  # gradients accumulate straight into the bucket buffer
        # the tensor whose backward gradient feeds segment i: the parameter itself, or its bf16
        # working copy (parallel/precision.py) when the parameter is an fp32 master
        self.srcs: List[torch.Tensor] = list(params)
        self.pending = len(params)
        self.fired = [False] * len(params)
        self.stolen: List[Optional[torch.Tensor]] = [None] * len(params)  # fresh grads awaiting the gather
        self.copy_later = set()  # stolen grads that need a layout copy, not the gather kernel
        self.handles = None
        self.ctx = None

    def reset(self):
        self.pending = len(self.params)
        self.fired = [False] * len(self.params)
        self.stolen = [None] * len(self.params)
        self.copy_later = set()
        self.handles = None
        self.ctx = None


class GraceEngine:
    """Owns the buckets, hooks, streams and in-flight handles of one model."""

    def __init__(self, params: Sequence[Tuple[str, torch.nn.Parameter]], grc: Communicator,
                 bucket_cap_mb: float = 64.0, backward_passes_per_step: int = 1, overlap: bool = True,
                 sparse_params: Sequence[str] = (), debug: Optional[bool] = None,
                 grad_sources: Optional[Dict[int, torch.Tensor]] = None,
                 group_collectives: Optional[bool] = None, watchdog=None, tail_bucket: bool = False):
        """``tail_bucket``: the model's first layer weight (its weight gradient is the LAST one
        backward produces -- e.g. ResNet's 7x7 stem on the side stream) gets a bucket of its own,
        exchanged last: under a split-graph capture the other buckets' exchange then overlaps that
        weight gradient (each bucket launch waits only for the side-stream work of its own
        parameters).  Per-tensor codecs give identical results with any bucketing."""
        from ..utils import debug as _dbg
        from .comm import GroupedComm

        self.grc = grc
        # one RCCL group per step for the buckets' collectives (GroupedComm) when nothing is to
        # be gained from issuing them early: no overlap with backward and more than one rank
        if group_collectives is None:
            group_collectives = (not overlap) and grc.comm.world_size > 1
        if group_collectives and not isinstance(grc.comm, GroupedComm):
            gc = GroupedComm(grc.comm)
            grc.comm = gc
            for part in (grc.compressor, grc.memory):
                if hasattr(part, "bind_comm"):
                    part.bind_comm(gc)
        self.grouped = isinstance(grc.comm, GroupedComm)
        # compressors with a step-level exchange (PowerSGD: one P and one Q all-reduce per step
        # for all buckets) defer it to step_flush(), called once every bucket is compressed
        self._step_flush = getattr(grc.compressor, "step_flush", None)
        if self._step_flush is not None and hasattr(grc.compressor, "enable_step_level"):
            grc.compressor.enable_step_level(True)
        # failure detection (parallel/launch.py Watchdog): every synchronize() tracks the step's
        # collectives and raises in the training thread if an earlier one missed its deadline;
        # RCCL async errors (peer death) are polled on the native comm
        self.watchdog = watchdog
        self.debug = _dbg.ExchangeChecker(getattr(grc, "comm", None)) if (
            debug if debug is not None else _dbg.enabled_from_env()) else None
        self.overlap = overlap
        self.backward_passes_per_step = backward_passes_per_step
        named = [(n, p) for n, p in params if p.requires_grad]
        if not named:
            raise ValueError("no trainable parameters")
        names = [n for n, _ in named]
        if len(set(names)) != len(names):
            raise ValueError("parameter names must be unique")
        unknown = set(sparse_params) - set(names)
        if unknown:
            raise ValueError(f"sparse_params not among the trainable parameters: {sorted(unknown)[:5]}")
        # parameters with sparse gradients (nn.Embedding(sparse=True)) bypass the buckets: their
        # (indices, values) are all-gathered uncompressed, as the reference does for TF
        # IndexedSlices (patch_files/horovod/tensorflow/__init__.py:62-73)
        self._sparse: Dict[int, Tuple[str, torch.nn.Parameter]] = {
            id(p): (n, p) for n, p in named if n in set(sparse_params)}
        self._sparse_pending: Dict[int, Tuple] = {}
        named = [(n, p) for n, p in named if id(p) not in self._sparse]
        if not named:
            raise ValueError("no dense trainable parameters")
        self.device = named[0][1].device
        cap = int(bucket_cap_mb * 1024 * 1024 / 4)
        groups: List[List[Tuple[str, torch.nn.Parameter]]] = []
        cur: List[Tuple[str, torch.nn.Parameter]] = []
        size = 0
        tail = named[:1] if (tail_bucket and named[0][1].dim() == 4 and len(named) > 1) else []
        for n, p in reversed(named[len(tail):]):  # backward order
            if cur and size + p.numel() > cap:
                groups.append(cur)
                cur, size = [], 0
            cur.append((n, p))
            size += p.numel()
        if cur:
            groups.append(cur)
        if tail:
            groups.append(tail)
        # deterministic bucket names (same on every rank and across restarts, so GRACE state
        # in checkpoints -- residuals, momenta, step counters -- maps back to its bucket)
        self.buckets: List[Bucket] = []
        for i, grp in enumerate(groups):
            sig = ";".join(f"{n}:{tuple(p.shape)}" for n, p in grp).encode()
            self.buckets.append(Bucket(f"grace.b{i}.{fnv1a64(sig):016x}", [p for _, p in grp], self.device))
        # gradients of fp32 masters may arrive on bf16 working copies (grad_sources: id(master) ->
        # working parameter, parallel/precision.py): hooks go on the tensor that gets the gradient
        self._where: Dict[int, Tuple[Bucket, int, torch.Tensor]] = {}
        for b in self.buckets:
            for i, (p, v) in enumerate(zip(b.params, b.views)):
                src = (grad_sources or {}).get(id(p), p)
                b.srcs[i] = src
                if src is not p:
                    src.grad = None
                self._where[id(src)] = (b, i, v)
        # producers of weight gradients may write straight into the bucket (ops/wgrad.py
        # grad_target): the parameter carries its view
        for b in self.buckets:
            for p, src, v in zip(b.params, b.srcs, b.views):
                if src is p:
                    p._grace_grad_view = v
        # the engine joins the weight-gradient side stream before it reads any gradient (bucket
        # launch / synchronize): its parameters may compute weight gradients there (ops/wgrad.py)
        _wgrad.mark_joinable([src for b in self.buckets for src in b.srcs])
        self._passes: Dict[int, int] = {}
        self._hooks = []
        self.stream = torch.cuda.Stream(self.device) if (self.device.type == "cuda" and overlap) else None
        for b in self.buckets:
            for src in b.srcs:
                self._hooks.append(src.register_post_accumulate_grad_hook(self._hook))
        for _, p in self._sparse.values():
            self._hooks.append(p.register_post_accumulate_grad_hook(self._sparse_hook))
        self.in_flight = 0
        self._paused = False
        self._grads_none = False

    # ------------------------------------------------------------------ backward hooks
    def pause(self):
        """Context manager: backward passes inside do not trigger the GRACE exchange (used while
        warming up / capturing graphed forward-backward callables)."""
        import contextlib

        @contextlib.contextmanager
        def _ctx():
            self._paused = True
            try:
                yield
            finally:
                self._paused = False
        return _ctx()

    def _hook(self, p: torch.Tensor):
        if self._paused:
            return
        b, idx, view = self._where[id(p)]
        cnt = self._passes.get(id(p), 0) + 1
        if cnt < self.backward_passes_per_step:
            self._passes[id(p)] = cnt
            return
        self._passes[id(p)] = 0
        if p.grad is not None and p.grad.is_sparse:
            raise RuntimeError(f"parameter {self._name_of(p)} produced a sparse gradient: pass its name in "
                               "sparse_params= (uncompressed sparse all-gather)")
        if p.grad is not None and p.grad.data_ptr() != view.data_ptr():
            # .grad was None before backward (zero_grad(set_to_none=True), or a bf16 working copy):
            # AccumulateGrad handed over its fresh gradient.  It is kept alive and copied into the
            # bucket by ONE gather launch when the bucket is complete (native); else copied here.
            if self._gatherable(p.grad, view):
                b.stolen[idx] = p.grad
            elif _wgrad.split_active(p.grad.device):
                # a split capture joins the side stream only at the bucket launch: copy then
                b.stolen[idx] = p.grad
                b.copy_later.add(idx)
            else:
                if p.grad.is_cuda:
                    _wgrad.join(torch.cuda.current_stream(p.grad.device))
                view.copy_(p.grad)
                if p is not b.params[idx]:
                    p.grad = None
                b.params[idx].grad = view
        if b.fired[idx]:
            raise RuntimeError(f"{b.name}: gradient of parameter {idx} produced twice before synchronize() -- "
                               "increase backward_passes_per_step or call synchronize()")
        b.fired[idx] = True
        b.pending -= 1
        if b.pending == 0 and not (self.device.type == "cuda" and _wgrad.split_active(self.device)):
            self._launch(b)  # (a split capture launches every bucket from synchronize, after its join)

    @staticmethod
    def _gatherable(g: torch.Tensor, view: torch.Tensor) -> bool:
        # same shape and strides as the (dense) bucket view -> same dense memory image
        # (strides of size-1 dims do not move memory: a 1x1 conv's channels_last gradient and its
        # contiguous bucket view are the same image)
        return (g.is_cuda and g.dtype in (torch.float32, torch.bfloat16) and g.shape == view.shape
                and all(a == b for a, b, n in zip(g.stride(), view.stride(), g.shape) if n > 1)
                and _native.native_on(g.device))

    def _gather(self, b: Bucket) -> None:
        """Copy the handed-over gradients into the bucket (one kernel per dtype and <= 120
        tensors; bf16 gradients of working copies are widened), then point the masters' .grad at
        the bucket views and release the fresh gradients (stream-ordered: safe to reuse)."""
        idx = [i for i, g in enumerate(b.stolen) if g is not None]
        if not idx:
            return
        for i in idx:
            if i in b.copy_later:
                b.views[i].copy_(b.stolen[i])
        for dt in (torch.float32, torch.bfloat16):
            sel = [i for i in idx if b.stolen[i].dtype == dt and i not in b.copy_later]
            if sel:
                _native.lib().gather_segments([b.stolen[i] for i in sel], [b.layout.offsets[i] for i in sel], b.flat)
        for i in idx:
            if self.stream is not None:
                b.stolen[i].record_stream(self.stream)
            if b.srcs[i] is not b.params[i]:
                b.srcs[i].grad = None
            b.params[i].grad = b.views[i]
            b.stolen[i] = None

    def _name_of(self, p) -> str:
        b, i, _ = self._where[id(p)]
        return f"{b.name}[{i}]"

    def _sparse_hook(self, p: torch.Tensor):
        if self._paused or p.grad is None:
            return
        cnt = self._passes.get(id(p), 0) + 1
        if cnt < self.backward_passes_per_step:
            self._passes[id(p)] = cnt
            return
        self._passes[id(p)] = 0
        self._launch_sparse(p)

    def _launch_sparse(self, p: torch.Tensor):
        from .comm import allgather_rows

        g = p.grad
        if not g.is_sparse:  # a dense gradient for a sparse-declared param: exchange as rows
            g = g.to_sparse(1)
        g = g.coalesce()
        comm = self.grc.comm
        wi, fi = allgather_rows(comm, g.indices().t(), async_op=True)
        wv, fv = allgather_rows(comm, g.values(), async_op=True)
        self._sparse_pending[id(p)] = (p, (wi, fi), (wv, fv), g.shape)
        self.in_flight += 1

    def _finish_sparse(self):
        W = self.grc.comm.world_size
        for pid in [i for i in self._sparse if i not in self._sparse_pending]:
            p = self._sparse[pid][1]
            if p.grad is not None:  # gradient exists but backward hook did not fire (paused)
                self._launch_sparse(p)
        for p, (wi, fi), (wv, fv), shape in self._sparse_pending.values():
            wi.wait()
            wv.wait()
            vals = fv()
            if self.grc.compressor.average and W > 1:
                vals = vals / W
            p.grad = torch.sparse_coo_tensor(fi().t(), vals, shape).coalesce()
        self._sparse_pending.clear()

    def _launch(self, b: Bucket):
        if b.handles is not None:
            raise RuntimeError(f"{b.name}: gradient computed twice before synchronize() -- increase "
                               "backward_passes_per_step or call synchronize()")
        if self.stream is not None:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            _wgrad.join(self.stream)  # weight gradients issued on the side stream (ops/wgrad.py)
            with torch.cuda.stream(self.stream):
                self._gather(b)
                b.handles, b.ctx = self.grc.send_step(b.flat, b.name)
        else:
            if self.device.type == "cuda":
                # (a split capture waits only for the side-stream work of this bucket's parameters)
                _wgrad.join(torch.cuda.current_stream(self.device), params=b.srcs)
            self._gather(b)
            b.handles, b.ctx = self.grc.send_step(b.flat, b.name)
        self.in_flight += 1

    # ------------------------------------------------------------------ step side
    def synchronize(self):
        """Finish every bucket (launching any that backward did not complete, e.g. unused
        parameters), wait for the collectives, decompress into the bucket buffers."""
        for b in self.buckets:
            if b.handles is None:
                for i, p in enumerate(b.params):  # no gradient this step (unused parameter)
                    if not b.fired[i]:
                        if self._grads_none:
                            b.views[i].zero_()
                        elif p.grad is not None and p.grad.data_ptr() != b.views[i].data_ptr():
                            if p.grad.is_cuda:
                                _wgrad.join(torch.cuda.current_stream(p.grad.device))
                            b.views[i].copy_(p.grad)
                        p.grad = b.views[i]
                self._launch(b)
        if self._step_flush is not None:
            if self.stream is not None:
                with torch.cuda.stream(self.stream):
                    self._step_flush()
            else:
                self._step_flush()
        if self.grouped:
            if self.stream is not None:
                with torch.cuda.stream(self.stream):
                    self.grc.comm.flush()
            else:
                self.grc.comm.flush()
        cur = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        if self.stream is not None:
            cur.wait_stream(self.stream)
            for b in self.buckets:
                _record_stream((b.handles, b.ctx), cur)
        for b in self.buckets:
            if hasattr(b.ctx, "out"):
                b.ctx.out = b.flat  # decompress straight into the gradient bucket
            out = self.grc.receive_step(b.handles, b.ctx)
            if out.data_ptr() != b.flat.data_ptr():
                b.flat.copy_(out.view(-1))
            if self.debug is not None:
                self.debug.check_bucket(b.name, b.flat)
            b.reset()
        if self._sparse:
            self._finish_sparse()
        self.in_flight = 0
        # device-side communication faults (host-mapped health words: no sync, capture-safe)
        _health.check()
        if self.watchdog is not None:
            self.watchdog.check()
            capturing = self.device.type == "cuda" and torch.cuda.is_current_stream_capturing()
            check = getattr(self.grc.comm, "check", None)
            if callable(check) and not capturing:  # a comm's check may query the device
                check()
            if self.device.type == "cuda" and not capturing:
                self.watchdog.track_stream("GRACE exchange")

    def abort_step(self):
        """Forget a partially launched step (e.g. a HIP-graph capture that raised mid-backward):
        handles, contexts, fired flags, handed-over gradients, pass counters, deferred
        collectives.  The engine is then ready for a fresh eager step."""
        for b in self.buckets:
            b.reset()
        self._passes.clear()
        self._sparse_pending.clear()
        if hasattr(self.grc.compressor, "_pending"):
            self.grc.compressor._pending = []
        if self.grouped:
            self.grc.comm._pending = []
        self.in_flight = 0

    def zero_grad(self, set_to_none: bool = True):
        """``set_to_none`` (default): .grad becomes None, AccumulateGrad hands its fresh gradient
        to the hook and one native gather launch per bucket copies them in when the bucket is
        complete.  ``False``: memset the buckets, AccumulateGrad adds into the bucket views
        (one add kernel per parameter)."""
        if self.in_flight:
            raise AssertionError("zero_grad() called with gradients still being communicated -- "
                                 "call synchronize()/step() first")
        self._grads_none = set_to_none
        for b in self.buckets:
            for p, src in zip(b.params, b.srcs):
                if src is not p:
                    src.grad = None  # working copies always hand over a fresh gradient
        if set_to_none:
            for b in self.buckets:
                for p in b.params:
                    p.grad = None
        else:
            for b in self.buckets:
                b.flat.zero_()
                for p, v in zip(b.params, b.views):
                    p.grad = v
        for _, p in self._sparse.values():
            p.grad = None

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for b in self.buckets:
            for p, v in zip(b.params, b.views):
                if getattr(p, "_grace_grad_view", None) is v:
                    del p._grace_grad_view
        _wgrad.mark_joinable([src for b in self.buckets for src in b.srcs], on=False)

    def state_dict(self):
        return {"grc": self.grc.state_dict()}

    def load_state_dict(self, sd):
        self.grc.load_state_dict(sd["grc"])
