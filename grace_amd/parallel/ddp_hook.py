"""GRACE as a ``torch.nn.parallel.DistributedDataParallel`` communication hook.

The reference predates DDP comm hooks (survey 2.12); its torch.distributed surface is the
per-parameter loop ``grc.step(p.grad, name)`` after backward
(/root/reference/examples/dist/CIFAR10-dawndist/core.py:203-206).  This is the north-star
integration: ``ddp.register_comm_hook(GraceHookState(grc), grace_comm_hook)`` and DDP's own
bucketing, backward overlap and gradient copy-back drive the GRACE pipeline, with the SAME
per-parameter semantics as that loop (Top-K keeps a per-tensor k, EF-Sign a per-tensor scale ...).

For each DDP bucket the hook (called from the autograd thread as soon as the bucket is ready):
  1. derives the bucket's per-parameter layout from ``bucket.gradients()`` (views into the
     bucket buffer).  When DDP left gaps between the views (alignment padding), the gradients
     are first packed into a dense buffer with that layout and unpacked afterwards -- never a
     silent fall-back to one whole-bucket segment.  The bucket's GRACE name is derived from its
     parameters, and when DDP re-buckets (it does after the first iteration) the per-element
     GRACE state of the old buckets -- residuals, momenta -- is re-homed parameter by parameter
     into the new ones, so error feedback carries over exactly as in the per-parameter loop;
  2. runs compress + the async collective on a side **compress stream** forked from the
     compute stream, and the decode/aggregate on a separate **decode stream** that waits for the
     collective: the next bucket's compress never queues behind this bucket's decode, so
     compress(i+1) overlaps collective(i) and both overlap the rest of backward;
  3. returns a ``torch.futures.Future`` carrying the decoded bucket (completed on the decode
     stream -- DDP's finaliser waits on its CUDA event, backward compute is never blocked).
"""
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..core import Communicator, register_layout
from ..ops.layout import SegmentLayout


def mark_ddp_params(params, defer: bool = False) -> None:
    """Immediate hook: weight gradients of these parameters are computed in line (ops/wgrad.py):
    DDP's reducer reads each gradient from its AccumulateGrad hook, during backward, on the
    current stream.  Deferred hook: they may run on the side stream, written INTO their bucket
    views (the reducer then finds aliases and reads nothing); ``flush`` joins the side stream
    before the exchange reads a bucket."""
    from ..ops import wgrad as _wg

    params = list(params)
    for p in params:
        p._grace_ddp = True
        p._grace_alias_grad = bool(defer)
    _wg.mark_joinable(params, on=bool(defer))


# DDP-managed weight gradients stay in line.  Side-stream weight gradients for stable DDP buckets
# were measured slower on the graphed ResNet-50 step (2384-2388 vs 2487-2488 img/s in line, host
# issue 10.2 vs 0.15 ms per step: the forked capture falls off HIP's packet-capture launch path;
# profiles/r4_ddp_surface.txt), so the reducer's mid-backward reads never race a side stream.


class GraceHookState:
    def __init__(self, grc: Communicator, name: str = "ddp", model: Optional[torch.nn.Module] = None,
                 defer: bool = False):
        """``model``: the DistributedDataParallel module the hook is registered on -- pass it so
        its parameters are marked before the first backward (otherwise they are marked by the
        hook's first call, and the first backward may compute weight gradients on a side stream
        that the reducer does not wait for).

        ``defer``: the hook hands DDP the bucket buffer itself as an already-completed result and
        queues the bucket; :meth:`flush` (call it after ``backward()``, before the optimizer
        step -- ``GraceDDPOptimizer`` does) runs the GRACE exchange of every queued bucket on the
        current stream, decoding in place into the buffers the parameters' gradients alias.  No
        overlap of the exchange with backward (as the engine without overlap), but weight
        gradients may run on the side stream, and the step can be captured as a split graph
        (parallel/graph.py): the first join is in ``flush``, on the capture stream."""
        self.grc = grc
        self.name = name
        self.defer = bool(defer)
        self.pending = []  # deferred buckets: (GradBucket buffer, GRACE name, packed index)
        if model is not None:
            mark_ddp_params(model.parameters(), defer=self.defer)
        # bucket index -> (layout, packed index or None, buffer numel, GRACE name, param signature)
        self.layouts: Dict[int, tuple] = {}
        self.streams: Dict[int, Tuple[torch.cuda.Stream, torch.cuda.Stream]] = {}
        self.packed_buckets = 0  # buckets that needed the pack/unpack path (padding)
        self.migrations = 0      # per-element state re-homed after a DDP re-bucketing
        # id(param) -> (GRACE bucket name, flat offset, numel, layout total) of its current bucket
        self._loc: Dict[int, Tuple[str, int, int, int]] = {}
        self._gen: Dict[int, int] = {}
        self._views: Dict[int, int] = {}  # bucket index -> buffer address its gradient targets point into
        self._stable = set()  # bucket indices whose buffer was seen unchanged on consecutive calls

    def layout_for(self, bucket) -> Tuple[str, Optional[torch.Tensor]]:
        """(registered layout name, None | int64 index of the packed elements in the buffer)."""
        idx = bucket.index()
        buf = bucket.buffer()
        params = bucket.parameters()
        sig = tuple(id(p) for p in params)
        mark_ddp_params(params, defer=self.defer)
        ent = self.layouts.get(idx)
        if ent is None or ent[2] != buf.numel() or ent[4] != sig:
            from ..ops.randomk import fnv1a64

            grads = bucket.gradients()
            lay = SegmentLayout.from_tensors(grads)
            es = buf.element_size()
            offs = [(g.data_ptr() - buf.data_ptr()) // es for g in grads]
            dense = all(o == lay.offsets[i] for i, o in enumerate(offs)) and lay.total == buf.numel()
            pidx = None
            if not dense:  # DDP padding between the views: pack per-parameter segments densely
                pidx = torch.cat([torch.arange(o, o + g.numel(), dtype=torch.int64) for o, g in zip(offs, grads)])
                pidx = pidx.to(buf.device)
                self.packed_buckets += 1
            # rank-invariant name (seeds of RandomK & co. must agree across ranks): bucket index,
            # shapes and the layout generation of that index (DDP re-buckets identically everywhere)
            self._gen[idx] = self._gen.get(idx, -1) + 1
            shapes = ";".join(f"{tuple(g.shape)}" for g in grads)
            key = f"{self.name}.b{idx}.{fnv1a64(shapes.encode()):016x}.g{self._gen[idx]}"
            register_layout(key, lay)
            self._migrate(key, params, lay)
            ent = (lay, pidx, buf.numel(), key, sig)
            self.layouts[idx] = ent
        if self._views.get(idx) == buf.data_ptr():
            if idx not in self._stable:
                # the same bucket buffer on two consecutive calls: DDP's one-time bucket rebuild
                # (after the first iteration) is behind us and the marked views stay valid -- from
                # now on side-stream weight gradients may be written into them (deferred hook)
                self._stable.add(idx)
                for p in params:
                    p._grace_view_stable = True
        else:  # new layout, or DDP rebuilt the same one
            self._stable.discard(idx)
            for p in params:
                p._grace_view_stable = False
            self._views[idx] = buf.data_ptr()
            # with gradient_as_bucket_view DDP makes each .grad a view of the bucket: mark those
            # views as the parameters' gradient targets, so weight-gradient producers
            # (ops/wgrad.py) write straight into the bucket and the reducer finds an alias
            # instead of copying
            for p, g in zip(params, bucket.gradients()):
                if p.grad is not None and p.grad.data_ptr() == g.data_ptr() and p.grad.shape == g.shape:
                    p._grace_grad_view = g
        return ent[3], ent[1]

    def _containers(self):
        """The name-keyed per-element state dicts of the memory and the compressor."""
        for obj in (self.grc.memory, self.grc.compressor):
            for v in list(vars(obj).values()):
                if isinstance(v, dict) and v and all(isinstance(k, str) for k in v):
                    yield v

    def _migrate(self, key: str, params, lay: SegmentLayout) -> None:
        """Re-home the per-element state of ``params`` from their previous buckets into ``key``."""
        moves = []
        for i, p in enumerate(params):
            old = self._loc.get(id(p))
            if old is not None and old[0] != key:
                moves.append((i, old))
            self._loc[id(p)] = (key, lay.offsets[i], lay.numels[i], lay.total)
        if not moves:
            return
        for d in self._containers():
            new = None
            for i, (oname, ooff, on, ototal) in moves:
                src = d.get(oname)
                if not isinstance(src, torch.Tensor) or src.numel() != ototal or on != lay.numels[i]:
                    continue
                if new is None:
                    new = d.get(key)
                    if not isinstance(new, torch.Tensor) or new.numel() != lay.total:
                        new = torch.zeros(lay.total, dtype=src.dtype, device=src.device)
                        d[key] = new
                new.view(-1)[lay.offsets[i]:lay.offsets[i] + on].copy_(src.reshape(-1)[ooff:ooff + on])
        self.migrations += 1

    def flush(self) -> None:
        """Run the GRACE exchange of every deferred bucket, in backward order, on the current
        stream: join the weight-gradient side stream, compress + collective + decode straight
        into the bucket buffer (every parameter's gradient aliases it)."""
        if not self.pending:
            return
        from ..ops import wgrad as _wg

        pend, self.pending = self.pending, []
        for buf, name, pidx in pend:
            if buf.is_cuda:
                _wg.join(torch.cuda.current_stream(buf.device))
            _exchange_into(self.grc, buf, name, pidx)

    def _streams(self, dev):
        st = self.streams.get(dev.index)
        if st is None:
            st = self.streams[dev.index] = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
        return st


def _record(obj, stream, depth=0):
    if depth > 6 or obj is None:
        return
    if isinstance(obj, torch.Tensor):
        if obj.is_cuda:
            obj.record_stream(stream)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _record(o, stream, depth + 1)
    elif isinstance(obj, dict):
        for o in obj.values():
            _record(o, stream, depth + 1)
    elif hasattr(obj, "__dict__") and not isinstance(obj, type):
        for o in vars(obj).values():
            _record(o, stream, depth + 1)


def _exchange_into(grc: Communicator, buf: torch.Tensor, name: str, pidx) -> None:
    """Synchronous GRACE step of one bucket on the current stream, result written into ``buf``."""
    g = buf if (pidx is None and buf.dtype == torch.float32) else \
        (buf.float() if pidx is None else buf.float().index_select(0, pidx))
    handles, ctx = grc.send_step(g, name)
    in_place = pidx is None and buf.dtype == torch.float32
    if in_place and hasattr(ctx, "out"):
        ctx.out = buf  # decode straight into the bucket (compress has consumed it)
    out = grc.receive_step(handles, ctx).reshape(-1)
    if pidx is None:
        if out.data_ptr() != buf.data_ptr():
            buf.copy_(out.view_as(buf))
    else:
        full = torch.zeros_like(buf)
        full.index_copy_(0, pidx, out.to(buf.dtype))
        buf.copy_(full)


def grace_comm_hook(state: GraceHookState, bucket: dist.GradBucket) -> torch.futures.Future[torch.Tensor]:
    buf = bucket.buffer()
    name, pidx = state.layout_for(bucket)
    grc = state.grc
    if state.defer:
        # the exchange runs in state.flush(); DDP gets its own buffer back (no copy-back), which
        # flush() then overwrites in place with the decoded gradient
        state.pending.append((buf, name, pidx))
        fut = torch.futures.Future(devices=[buf.device]) if buf.is_cuda else torch.futures.Future()
        fut.set_result(buf)
        return fut

    def packed(t):
        g = t if t.dtype == torch.float32 else t.float()
        return g if pidx is None else g.index_select(0, pidx)

    def unpacked(out):
        out = out.reshape(-1)
        if pidx is None:
            return out.to(buf.dtype).view_as(buf)
        full = torch.zeros_like(buf)
        full.index_copy_(0, pidx, out.to(buf.dtype))
        return full

    if not buf.is_cuda:
        out = grc.step(packed(buf), name)
        fut = torch.futures.Future()
        fut.set_result(unpacked(out))
        return fut
    dev = buf.device
    from ..ops import wgrad as _wg

    cs, ds = state._streams(dev)
    cur = torch.cuda.current_stream(dev)
    cs.wait_stream(cur)

    _wg.join(cs)  # any side-stream weight gradient issued so far (none for DDP-managed weights)
    with torch.cuda.stream(cs):
        g = packed(buf)
        handles, ctx = grc.send_step(g, name)  # compress + async collective (comm stream or inline)
    ds.wait_stream(cs)  # decode after this bucket's compress/issue; the collective is waited on inside
    fut = torch.futures.Future(devices=[dev])
    in_place = pidx is None and buf.dtype == torch.float32 and g.data_ptr() == buf.data_ptr()
    with torch.cuda.stream(ds):
        # the payload tensors and the context's per-call tensors cross to the decode stream
        # (not a deep walk of the context: its layout holds long-lived cached device tables)
        _record(handles, ds)
        _record(getattr(ctx, "extra", None), ds)
        _record(getattr(ctx, "out", None), ds)
        if in_place and hasattr(ctx, "out"):
            ctx.out = buf  # decode straight into the bucket (compress has consumed it)
        out = grc.receive_step(handles, ctx)
        if in_place:
            # hand DDP its OWN bucket buffer: the reducer then finds every parameter's gradient
            # already aliasing its bucket view; any other tensor makes it copy the result into
            # each parameter's gradient, one copy kernel per parameter (161 for ResNet-50)
            if out.data_ptr() != buf.data_ptr():
                buf.copy_(out.reshape(-1).view_as(buf))
            out = buf
        else:
            out = unpacked(out)
        buf.record_stream(ds)
        g.record_stream(ds)
        fut.set_result(out)
    return fut


class GraceDDPOptimizer:
    """``optimizer`` whose ``step()`` first runs the deferred GRACE exchange of a
    ``GraceHookState(defer=True)`` (``state.flush()``), then the wrapped optimizer's step.

        ddp = DistributedDataParallel(model, gradient_as_bucket_view=True)
        state = GraceHookState(grc, model=ddp, defer=True)
        ddp.register_comm_hook(state, grace_comm_hook)
        opt = GraceDDPOptimizer(torch.optim.SGD(ddp.parameters(), lr=0.1), state)
    """

    def __init__(self, optimizer, state: GraceHookState):
        self.optimizer = optimizer
        self.state = state

    def step(self, closure=None):
        self.state.flush()
        return self.optimizer.step(closure) if closure is not None else self.optimizer.step()

    def zero_grad(self, set_to_none: bool = True):
        if self.state.pending:
            raise AssertionError("zero_grad() with deferred GRACE buckets pending -- call step() first")
        self.optimizer.zero_grad(set_to_none=set_to_none)

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    def state_dict(self):
        return self.optimizer.state_dict()

    def load_state_dict(self, sd):
        self.optimizer.load_state_dict(sd)
