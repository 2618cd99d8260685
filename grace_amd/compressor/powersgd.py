"""PowerSGD -- rank-r power-iteration compression (Vogels et al., NeurIPS 2019).

Reference: /root/reference/grace_dl/dist/compressor/powersgd.py:7-65 -- for every >=2-D tensor
M (n x m): Q (m x r) ~ N(0,1) orthogonalised, P = M Q, all_reduce(P)/W, orthogonalise(P),
Q = M^T P, all_reduce(Q)/W, decompress P Q^T; 1-D tensors are sent uncompressed; the payload of
matrices is empty (all communication happens inside compress).

Fixes / design (survey 2.14 #4, #5, #7): the real world size divides P and Q (the reference's
default world_size=1 makes the result W x too large); Q is drawn from a seed shared by all
ranks (name, step) so every rank multiplies by the SAME Q; warm start (reuse last Q, the
paper's recipe) is available as ``warm_start=True``.  For a flat bucket all matrices' P live in
ONE buffer and all Q in another, so a whole bucket costs exactly two all-reduces; the 1-D
segments travel through the communicator (Allreduce).  PowerSGD is only meaningful with the
Allreduce communicator (Allgather would silently zero matrices in the reference).

MI355X kernels (csrc/kernels/powersgd.hip): P = M Q and Q = M^T P as batched tall-skinny
fp32 MFMA GEMMs (v_mfma_f32_32x32x2_f32 / 16x16x4, all matrices of the bucket in ONE launch
each), batched LDS-resident Gram-Schmidt (one workgroup per matrix), and decompress
P Q^T fused with the residual update.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Tuple

import torch

from ..ops import powersgd as PS
from ..ops.randomk import fnv1a64, mix_step
from ._base import BucketCompressor, Ctx


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
        return self._power(x, x, name, ctx, plan), ctx

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
        # x (matrix segments) lands in r; 1-D segments of x equal g (their residual is zero)
        vec = self._power(g, r, name, ctx, plan, comp_r=r if valid else None, xout=r)
        ctx.extra["resid"] = r
        return vec, ctx

    def _power(self, x, x_after, name, ctx, plan, comp_r=None, xout=None):
        """One power iteration for every matrix of the bucket.  ``x`` feeds the first product
        (compensated on the fly when ``xout`` is given, which then holds x); ``x_after`` is
        what the second product reads."""
        W = self.world_size or 1
        step, step_t = self.advance(name, x.device)
        q = self.q_memory.get(name) if self.warm_start else None
        if q is None or q.numel() != plan.q_total:
            # identical on every rank (no rank in the seed); the device step counter keeps a fresh
            # Q per HIP-graph replay when warm_start is off
            seed = fnv1a64(name.encode())
            q = PS.randn_shared(plan.q_total, seed if step_t is not None else mix_step(seed, step), x.device,
                                step=step_t)
            # The reference orthogonalises this fresh Gaussian Q (dist/compressor/powersgd.py:43).  That cannot
            # change the result: MGS gives Q R^-1 with R upper triangular, so P = M Q R^-1 = P R^-1
            # and the orthonormal factor of P R^-1 is that of P -- orthogonalize(P) below yields the
            # same P-hat, hence the same Q = M^T P-hat and P-hat Q^T (up to rounding; a Gaussian Q is
            # well conditioned).  Skipped: it was a 400 KB single-workgroup pass per step for
            # VGG-16's 25088 x 4 Q.  (A warm-start Q is used as is, as in the reference.)
        p = PS.mq(x, q, plan, comp_r=comp_r, xout=xout)  # P = M Q for every matrix (one launch)
        if self.comm is not None and W > 1:
            self.comm.all_reduce(p)
        if W > 1:
            p.div_(W)
        PS.orthogonalize(p, plan, which="p")
        q = PS.mtp(x_after, p, plan)  # Q = M^T P
        if self.comm is not None and W > 1:
            self.comm.all_reduce(q)
        if W > 1:
            q.div_(W)
        if self.warm_start:
            self.q_memory[name] = q
        ctx.extra.update(plan=plan, p=p, q=q)
        vec = PS.gather_vectors(x, plan)  # 1-D segments, sent through the communicator
        return [vec] if vec.numel() else []

    def _decompress(self, tensors, ctx, vec_scale: float):
        plan = ctx.extra["plan"]
        dev = tensors[0].device if tensors else ctx.extra["p"].device
        if plan.n_mat == 0:
            (v,) = tensors
            out = v * vec_scale if vec_scale != 1.0 else v
            return self.finish(out.reshape(-1), ctx)
        out = self.out_buffer(ctx, dev)
        # fused path: the residual buffer holds x; this pass also leaves r = x - P Q^T there
        PS.pqt(ctx.extra["p"], ctx.extra["q"], plan, out, resid=ctx.extra.pop("resid", None))
        if tensors:
            PS.scatter_vectors(tensors[0], plan, out, vec_scale)
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
