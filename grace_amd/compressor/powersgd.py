"""PowerSGD -- rank-r power-iteration compression (Vogels et al., NeurIPS 2019).

Reference: /root/reference/grace_dl/dist/compressor/powersgd.py:7-65 -- for every >=2-D tensor
M (n x m): Q (m x r) ~ N(0,1) orthogonalised, P = M Q, all_reduce(P)/W, orthogonalise(P),
Q = M^T P, all_reduce(Q)/W, decompress P Q^T; 1-D tensors are sent uncompressed; the payload of
matrices is empty (all communication happens inside compress).

Fixes / design (survey 2.14 #4, #5, #7): the real world size divides the result (the
reference's default world_size=1 makes it W x too large); Q is drawn from a seed shared by all
ranks (name, step) so every rank multiplies by the SAME Q; warm start (reuse last Q, the
paper's recipe) is available as ``warm_start=True``.

Collectives: SURVEY 2.11 prescribes "2 allreduces per step for the whole model (flat P, flat Q)".
Under :class:`~grace_amd.parallel.engine.GraceEngine` (``step_level``) every bucket's P lands in
its slice of ONE step-level P arena during backward; ``step_flush`` (called by the engine once
all buckets are compressed) issues ONE P all-reduce, orthonormalises every P, writes every
Q = M^T P into ONE Q arena and issues ONE Q all-reduce -- two matrix collectives per step however
many buckets the model has (the reference issues two per matrix,
/root/reference/grace_dl/dist/compressor/powersgd.py:45-52).  No division kernels: the
orthonormalisation is scale invariant, so P is orthonormalised as the SUM over ranks, and the
1/W of Q is folded into the P Q^T decompress pass (``ps_pqt`` ``scale``).  The manual
``grc.step`` path (one tensor at a time) runs the same exchange immediately.  1-D segments travel
through the communicator (Allreduce).  PowerSGD is only meaningful with the Allreduce
communicator (Allgather would silently zero matrices in the reference).

MI355X kernels (csrc/kernels/powersgd.hip): P = M Q and Q = M^T P as bandwidth-shaped VALU
tall-skinny products (16-B loads, every matrix of the bucket in ONE launch each; MFMA tiles were
measured at < 2 % matrix-core busy for r <= 4 -- the products are HBM-bound at ~2r FLOP per
loaded element), the Gram matrix of the orthonormalisation on MFMA (v_mfma_f32_16x16x4_f32) for
r > 4, register-resident MGS for r <= 4, and decompress P Q^T fused with the residual update.
"""
from __future__ import annotations

import torch

from ..ops import powersgd as PS
from ..ops.randomk import fnv1a64, mix_step
from ._base import BucketCompressor, Ctx

# GRACE_POWERSGD_DEFER_RESID=0: the residual update r = x - P Q^T stays in the decompress pass
# (reads and rewrites the residual); default: deferred into the next step's P = M Q pass
_DEFER_RESID = __import__("os").environ.get("GRACE_POWERSGD_DEFER_RESID", "1") == "1"


class PowerSGDCompressor(BucketCompressor):
    allreduce_compatible = True
    _state_attrs = ("steps", "q_memory")

    def __init__(self, rank: int = 1, use_memory: bool = False, world_size: int | None = None,
                 warm_start: bool | None = None):
        super().__init__()
        self.rank_r = int(rank)
        self.warm_start = bool(use_memory if warm_start is None else warm_start)
        self.world_size = world_size
        self.q_memory = {}
        self.comm = None
        # step-level batching (GraceEngine): deferred buckets of the current step and the
        # P / Q arenas ({"key", "p", "q", "off": name -> (p_off, q_off)})
        self.step_level = False
        self._pending = []
        self._arena = None
        self.matrix_collectives = 0  # matrix all-reduces issued (tests / monitoring)
        self._pq_prev = {}  # name -> [P | Q] of the last step (deferred residual), persistent
        self._q_cleared = False  # the step's first P-clearing launch also cleared the Q arena

    def enable_step_level(self, on: bool = True):
        """Defer the P/Q exchange of every bucket to :meth:`step_flush` (called by the engine)."""
        self.step_level = bool(on)

    def bind_comm(self, comm):
        super().bind_comm(comm)
        if self.world_size is None:
            self.world_size = comm.world_size

    def _plan(self, ctx: Ctx) -> PS.Plan:
        return PS.plan_for(ctx.layout, self.rank_r)

    def compress(self, tensor, name):
        ctx = self.ctx(tensor, name)
        plan = self._plan(ctx)
        if plan.n_mat == 0:  # no matrix: reference passes 1-D tensors through
            ctx.extra["plan"] = plan
            return [self.flat(tensor)], ctx
        x = self.flat(tensor)
        # not deferred: a non-fused memory's update() decompresses right after compress
        return self._power(x, x, name, ctx, plan, defer=False), ctx

    def fused_compress(self, tensor, name, memory):
        """PowerSGDMemory fused into the kernels: the compensate x = r + g is computed while
        staging M for P = M Q (and stored into the residual buffer), and the residual update
        r = x - P Q^T happens in the decompress pass that writes P Q^T anyway -- 7 passes
        over the bucket instead of 10 (axpby, MQ, M^T P, P Q^T twice, x - dec)."""
        from ..memory.powersgd import PowerSGDMemory

        if type(memory) is not PowerSGDMemory:
            return None
        ctx = self.ctx(tensor, name)
        plan = self._plan(ctx)
        if plan.n_mat == 0:
            return None
        g = self.flat(tensor)
        if not memory.warm_start:
            self.q_memory.pop(name, None)
        rs = memory.residuals.get(name)
        valid = rs is not None and rs.numel() == g.numel() and rs.dtype == torch.float32 and rs.is_contiguous()
        if not valid:
            # 1-D segments keep a zero residual (reference: no error feedback for them)
            rs = torch.zeros(tensor.shape, dtype=torch.float32, device=g.device)
            memory.residuals[name] = rs
        r = rs.view(-1)
        # deferred residual of the previous step (r holds its M): formed inside this P = M Q pass
        lz = memory.lazy.get(name)
        lazy = None
        if lz is not None and valid and lz[3] is plan:
            lazy = (lz[0], lz[1], lz[2])
            del memory.lazy[name]
        elif lz is not None:
            # cannot be fused into this pass (re-planned layout, same numel): apply it now, so r
            # is the true residual M - s P Q^T and not the previous M; a residual
            # that is being reset (not valid) drops it with the buffer
            if valid:
                memory.materialize(name)
            else:
                del memory.lazy[name]
        # x (matrix segments) lands in r; 1-D segments of x equal g (their residual is zero)
        vec = self._power(g, r, name, ctx, plan, comp_r=r if valid else None, xout=r, defer=self.step_level,
                          lazy=lazy)
        ctx.extra["resid"] = r
        if _DEFER_RESID and g.is_cuda:
            ctx.extra["lazy_mem"] = memory
            ctx.extra["name"] = name
        return vec, ctx

    def _arena_slice(self, name, plan):
        a = self._arena
        if a is None or name not in a["off"]:
            return None
        po, qo = a["off"][name]
        if po + plan.p_total > a["p"].numel():
            return None
        return a["p"][po:po + plan.p_total]

    def _power(self, x, x_after, name, ctx, plan, comp_r=None, xout=None, defer=False, lazy=None):
        """P = M Q for every matrix of the bucket (into the step-level P arena when batching);
        the P/Q collectives run now (manual path) or in :meth:`step_flush`.  ``x`` feeds the
        first product (compensated on the fly when ``xout`` is given, which then holds x);
        ``x_after`` is what the second product reads."""
        native = PS._native.use_native(x)
        # native: the P = M Q launch advances the device step counter (post-bump, no add kernel)
        step, step_t = self.advance(name, x.device, post=native)
        sl = p_out = self._arena_slice(name, plan) if defer else None
        if native and p_out is None:
            p_out = torch.empty(plan.p_total, dtype=torch.float32, device=x.device)
        zero = p_out
        a = self._arena
        if native and sl is not None and not self._pending and not self.warm_start and a["off"][name][0] == 0:
            # the step's first bucket: [Q arena | P arena] is one buffer and this bucket's P slice
            # leads the P arena, so the launch that clears P clears the Q arena too (no memset
            # before the step's M^T P launch)
            zero = a["qp"][:a["q"].numel() + plan.p_total]
            self._q_cleared = True
        zeroed = False
        q = self.q_memory.get(name) if self.warm_start else None
        if q is None or q.numel() != plan.q_total:
            # identical on every rank (no rank in the seed); the device step counter keeps a fresh
            # Q per HIP-graph replay when warm_start is off
            seed = fnv1a64(name.encode())
            # the same launch clears P for the accumulating P = M Q launch (no memset)
            q = PS.randn_shared(plan.q_total, seed if step_t is not None else mix_step(seed, step), x.device,
                                step=step_t, zero=zero if native else None)
            zeroed = native
        elif zero is not p_out:
            self._q_cleared = False
            # The reference orthogonalises this fresh Gaussian Q (dist/compressor/powersgd.py:43).  That cannot
            # change the result: MGS gives Q R^-1 with R upper triangular, so P = M Q R^-1 = P R^-1
            # and the orthonormal factor of P R^-1 is that of P -- orthogonalize(P) below yields the
            # same P-hat, hence the same Q = M^T P-hat and P-hat Q^T (up to rounding; a Gaussian Q is
            # well conditioned).  Skipped: it was a 400 KB single-workgroup pass per step for
            # VGG-16's 25088 x 4 Q.  (A warm-start Q is used as is, as in the reference.)
        # 1-D segments, sent through the communicator: packed by the P = M Q launch (native)
        vec = torch.empty(plan.v_total, dtype=torch.float32, device=x.device) if native else None
        p = PS.mq(x, q, plan, comp_r=comp_r, xout=xout, out=p_out, lazy=lazy, zeroed=zeroed,
                  bump=step_t if native else None, vec=vec)  # P = M Q, every matrix, one launch
        ctx.extra.update(plan=plan, p=p)
        if vec is None:
            vec = PS.gather_vectors(x, plan)
        entry = (name, x_after, ctx)
        if defer:
            self._pending.append(entry)
        else:
            self._exchange([entry])
        return [vec] if vec.numel() else []

    def step_flush(self):
        """The step's P/Q exchange for every deferred bucket: one P all-reduce, one Q
        all-reduce.  Every rank calls it at the same point (the engine's synchronize)."""
        pend, self._pending = self._pending, []
        if pend:
            self._exchange(pend, arena=True)

    def _build_arena(self, entries):
        dev = entries[0][2].extra["p"].device
        off, po, qo = {}, 0, 0
        for name, _, ctx in entries:
            plan = ctx.extra["plan"]
            off[name] = (po, qo)
            po += plan.p_total
            qo += plan.q_total
        key = tuple((name, ctx.extra["plan"].p_total, ctx.extra["plan"].q_total) for name, _, ctx in entries)
        # every bucket's matrices over the whole P arena: ONE orthonormalisation launch per step
        # (one per bucket cost ~10-20 us each of single-workgroup-per-matrix latency)
        mats = []
        for name, _, ctx in entries:
            bpo, bqo = off[name]
            plan = ctx.extra["plan"]
            mats += [(xo, n, m, r, mpo + bpo, mqo + bqo) for (xo, n, m, r, mpo, mqo) in plan.mats]
        orth = PS.Plan(self.rank_r, mats, [], po, qo, 0)
        qp = torch.empty(qo + po, dtype=torch.float32, device=dev)  # [Q arena | P arena]
        self._arena = {"key": key, "off": off, "qp": qp, "p": qp[qo:], "q": qp[:qo], "orth": orth,
                       "T": torch.empty(max(1, len(mats)) * 16, dtype=torch.float32, device=dev)}

    def _merged_mtp(self, entries):
        """(base tensor, plan) of one Q = M^T P launch over every bucket of the arena: each
        matrix's x offset is taken relative to the lowest bucket address (the buckets are separate
        allocations of one device; the kernel addresses them from that base).  None when it does
        not apply (CPU, misaligned or mixed-device buffers)."""
        xs = [x for _, x, _ in entries]
        if not all(PS._native.use_native(x) and x.dtype == torch.float32 and x.is_contiguous()
                   and x.device == xs[0].device for x in xs):
            return None
        ptrs = tuple(x.data_ptr() for x in xs)
        if any(p_ % 16 for p_ in ptrs):
            return None
        a = self._arena
        cached = a.get("mtp")
        if cached is not None and cached[0] == ptrs:
            return cached[1], cached[2]
        bi = min(range(len(xs)), key=lambda i: ptrs[i])
        base = xs[bi]
        mats = []
        for (name, _, ctx), ptr in zip(entries, ptrs):
            bpo, bqo = a["off"][name]
            d = (ptr - ptrs[bi]) // 4
            mats += [(xo + d, n, m, r, mpo + bpo, mqo + bqo) for (xo, n, m, r, mpo, mqo) in ctx.extra["plan"].mats]
        plan_all = PS.Plan(self.rank_r, mats, [], a["p"].numel(), a["q"].numel(), 0)
        a["mtp"] = (ptrs, base, plan_all)
        return base, plan_all

    def _exchange(self, entries, arena: bool = False):
        W = self.world_size or 1
        comm = self.comm if (self.comm is not None and W > 1) else None
        if arena:
            key = tuple((name, ctx.extra["plan"].p_total, ctx.extra["plan"].q_total) for name, _, ctx in entries)
            if self._arena is None or self._arena["key"] != key:
                self._build_arena(entries)  # first step (or a changed bucket set): re-home P
                self._q_cleared = False  # (a clear, if any, went to the previous arena)
            a = self._arena
            p_all, q_all = a["p"], a["q"]
            for name, _, ctx in entries:
                po, qo = a["off"][name]
                plan = ctx.extra["plan"]
                pv = p_all[po:po + plan.p_total]
                if ctx.extra["p"].data_ptr() != pv.data_ptr():
                    pv.copy_(ctx.extra["p"])
                    ctx.extra["p"] = pv
                ctx.extra["q"] = q_all[qo:qo + plan.q_total]
        else:
            ((name, _, ctx),) = entries
            p_all = ctx.extra["p"]
            q_all = torch.empty(ctx.extra["plan"].q_total, dtype=torch.float32, device=p_all.device)
            ctx.extra["q"] = q_all
        if comm is not None:
            comm.all_reduce(p_all)  # SUM over ranks: the orthonormalisation is scale invariant
            self.matrix_collectives += 1
        cleared, self._q_cleared = self._q_cleared, False
        merged = self._merged_mtp(entries) if arena else None
        if merged is not None and self.rank_r <= 4:
            # ONE launch for the whole step: Q = M^T P of every bucket (the small buckets' tiles fill
            # in beside the big ones) with the orthonormalising transforms T of every P computed by
            # extra workgroups of the same launch; P stays as reduced, and P T / Q T are formed by
            # the decompress launches (the Gram work hides under the bandwidth-bound product)
            base, plan_all = merged
            if not cleared:
                q_all.zero_()
            T = self._arena["T"]
            PS.mtp_gram(base, p_all, plan_all, q_all, T)
            i = 0
            for _, _, ctx in entries:
                k = ctx.extra["plan"].n_mat
                ctx.extra["T"] = T[16 * i:16 * (i + k)]
                i += k
        else:
            if arena:
                # all buckets, one launch -- which also clears the Q arena for the M^T P launches
                PS.orthogonalize(p_all, self._arena["orth"], which="p", zero=None if cleared else q_all)
            else:
                for _, _, ctx in entries:
                    PS.orthogonalize(ctx.extra["p"], ctx.extra["plan"], which="p")
            if merged is not None:
                base, plan_all = merged
                PS.mtp(base, p_all, plan_all, out=q_all, zeroed=True)
            else:
                for _, x_after, ctx in entries:
                    PS.mtp(x_after, ctx.extra["p"], ctx.extra["plan"], out=ctx.extra["q"], zeroed=arena)  # Q = M^T P
        if comm is not None:
            comm.all_reduce(q_all)  # SUM; the 1/W is applied inside the P Q^T pass
            self.matrix_collectives += 1
        for name, _, ctx in entries:
            ctx.extra["q_scale"] = 1.0 / W
            if self.warm_start:
                self.q_memory[name] = ctx.extra["q"]  # scale is irrelevant: P = M Q is re-orthonormalised

    def _decompress(self, tensors, ctx, vec_scale: float):
        plan = ctx.extra["plan"]
        dev = tensors[0].device if tensors else ctx.extra["p"].device
        if plan.n_mat == 0:
            (v,) = tensors
            out = v * vec_scale if vec_scale != 1.0 else v
            return self.finish(out.reshape(-1), ctx)
        out = self.out_buffer(ctx, dev)
        if "q" not in ctx.extra:
            raise RuntimeError("PowerSGD: decompress before the step's P/Q exchange (call step_flush())")
        resid = ctx.extra.pop("resid", None)
        mem = ctx.extra.pop("lazy_mem", None)
        scale = ctx.extra.get("q_scale", 1.0)
        # the 1-D segments go back into out inside the P Q^T launch
        vec = tensors[0] if tensors and tensors[0].numel() == plan.v_total else None
        if vec is None and tensors:
            raise RuntimeError(f"PowerSGD: 1-D payload of {tensors[0].numel()} elements, plan has {plan.v_total}")
        if mem is not None and resid is not None:
            # deferred residual: the residual buffer keeps x, and (P, Q, scale) go to the memory
            # for the next step's P = M Q pass -- as copies in persistent per-name buffers: the
            # next P = M Q pass rewrites the step-level P arena slice while reading the previous P,
            # and a HIP graph replays fixed pointers (the manual path's P / Q are fresh tensors)
            name = ctx.extra["name"]
            prev = self._pq_prev.get(name)
            dev = ctx.extra["p"].device
            if prev is None or prev.numel() != plan.p_total + plan.q_total or prev.device != dev:
                prev = self._pq_prev[name] = torch.empty(plan.p_total + plan.q_total, dtype=torch.float32, device=dev)
            pp, qp = prev[:plan.p_total], prev[plan.p_total:]
            # the copies are stored by the decompress launch itself (it reads P and Q anyway)
            PS.pqt(ctx.extra["p"], ctx.extra["q"], plan, out, resid=None, scale=scale, save=(pp, qp), vec=vec,
                   vec_scale=vec_scale, T=ctx.extra.pop("T", None))
            mem.lazy[name] = (pp, qp, scale, plan)
        else:
            # fused eager form / unfused: the residual buffer holds x; this pass leaves r = x - P Q^T
            PS.pqt(ctx.extra["p"], ctx.extra["q"], plan, out, resid=resid, scale=scale, vec=vec, vec_scale=vec_scale,
                   T=ctx.extra.pop("T", None))
        return self.finish(out, ctx)

    def decompress(self, tensors, ctx):
        return self._decompress(tensors, ctx, 1.0)

    def decompress_reduced(self, tensors, ctx, world_size):
        return self._decompress(tensors, ctx, 1.0 / world_size if self.average else 1.0)

    def decompress_aggregate(self, per_rank, ctx, world_size):
        # Allgather/Broadcast: matrices are already averaged inside compress; sum the 1-D parts
        if not per_rank[0]:
            return self._decompress([], ctx, 1.0)
        vec = per_rank[0][0].clone()
        for p in per_rank[1:]:
            vec.add_(p[0])
        return self._decompress([vec], ctx, 1.0 / world_size if self.average else 1.0)
