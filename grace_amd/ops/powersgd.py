"""PowerSGD building blocks over a flat bucket (native: csrc/kernels/powersgd.hip).

A :class:`Plan` describes every matrix segment of a bucket (rows n, cols m, rank r and its
offsets into the flat gradient, the flat P buffer [sum n*r] and the flat Q buffer [sum m*r]),
plus the 1-D segments that bypass the low-rank path.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from . import _native
from .layout import SegmentLayout


# ps_mq column strip (power of two, 512..65536) and the ps_mtp workgroup target per matrix
# (row strips x 1024-column blocks): tuning knobs, GRACE_PS_MQ_COLS / GRACE_PS_MTP_WG
_MQ_COLS_SET = "GRACE_PS_MQ_COLS" in os.environ
_MQ_COLS = int(os.environ.get("GRACE_PS_MQ_COLS", "2048"))
# workgroups a P = M Q launch should have before its column strips stop shrinking
_MIN_WG = int(os.environ.get("GRACE_PS_MIN_WG", "4096"))
# rows per P Q^T workgroup strip (1..32)
_PQT_ROWS = int(os.environ.get("GRACE_PS_PQT_ROWS", "32"))
if not 1 <= _PQT_ROWS <= 32:
    raise ValueError("GRACE_PS_PQT_ROWS must be in [1, 32]")
_MTP_WG = int(os.environ.get("GRACE_PS_MTP_WG", "1024"))
if _MQ_COLS < 512 or _MQ_COLS > 65536 or _MQ_COLS & (_MQ_COLS - 1):
    raise ValueError("GRACE_PS_MQ_COLS must be a power of two in [512, 65536]")


@dataclass
class Plan:
    rank: int
    mats: List[Tuple[int, int, int, int, int, int]]  # (x_off, n, m, r, p_off, q_off)
    vecs: List[Tuple[int, int, int]]  # (x_off, numel, vec_off)
    p_total: int
    q_total: int
    v_total: int
    _dev: Dict[str, dict] = field(default_factory=dict, repr=False)

    @property
    def n_mat(self) -> int:
        return len(self.mats)

    def _mq_blocks(self, cs: int) -> int:
        return sum(-(-n // 16) * -(-m // cs) for (_, n, m, _, _, _) in self.mats)


    def tables(self, device):
        key = str(device)
        t = self._dev.get(key)
        if t is None:
            # work tables of csrc/kernels/powersgd.hip (ps_mq: 16 rows x 2048 columns; ps_mtp:
            # 1024 / 256 columns x per-matrix row strips; ps_pqt: 32 rows x 1024 / 256 columns)
            t0, t1, tp = [], [], []
            cs, prs = _MQ_COLS, _PQT_ROWS
            if not _MQ_COLS_SET:
                # P = M Q runs faster with more workgroups: shorter column strips until the launch
                # has _MIN_WG of them (VGG-16 fc6: 248 -> 234 us at 1024 columns; the P Q^T
                # launches measured SLOWER with shorter row strips: 70 -> 75 us -- they stay at 32)
                while cs > 512 and self._mq_blocks(cs) < _MIN_WG:
                    cs //= 2
            lg = cs.bit_length() - 1
            for i, (xo, n, m, r, po, qo) in enumerate(self.mats):
                cb = 1024 if (xo % 4 == 0 and m % 4 == 0) else 256
                for rb in range((n + 15) // 16):
                    for sidx in range((m + cs - 1) // cs):
                        t0.append((i, rb, sidx | (lg << 24)))
                # ps_mtp: 1024 (16-B path) / 256 (4-B path) column blocks; rows split into strips of a
                # multiple of 32 rows so that the matrix yields >= ~1024 workgroups (too few waves
                # left the product latency bound)
                ncb = (m + cb - 1) // cb
                n32 = (n + 31) // 32
                strips = max(1, min(n32, -(-_MTP_WG // ncb)))
                per = -(-n32 // strips)
                for c in range(ncb):
                    for s0 in range(0, n32, per):
                        t1.append((i, c, (s0 << 16) | min(per, n32 - s0)))
                for r0 in range(0, n, prs):
                    for c in range((m + cb - 1) // cb):
                        tp.append((i, r0, c | (min(prs, n - r0) << 20)))

            def it(lst):
                return torch.tensor(lst, dtype=torch.int32, device=device).view(-1) if lst else \
                    torch.empty(0, dtype=torch.int32, device=device)

            # Gram tiles of 256 rows over each P_i (n rows) and Q_i (m rows)
            gt = {"p": [], "q": []}
            gtb = {"p": [0], "q": [0]}
            for (xo, n, m, r, po, qo) in self.mats:
                for which, ln in (("p", n), ("q", m)):
                    for tix in range((ln + 255) // 256):
                        gt[which].append((len(gtb[which]) - 1, tix))
                    gtb[which].append(len(gt[which]))
            vec_idx = [i for (xo, n, vo) in self.vecs for i in range(xo, xo + n)]
            t = {
                "mat": torch.tensor([list(m) for m in self.mats] or [[0] * 6], dtype=torch.int64,
                                    device=device).contiguous(),
                "tiles0": it(t0),
                "tiles1": it(t1),
                "tilesp": it(tp),
                "gt_p": it(gt["p"]), "gtb_p": it(gtb["p"]),
                "gt_q": it(gt["q"]), "gtb_q": it(gtb["q"]),
                "vec_idx": torch.tensor(vec_idx, dtype=torch.int64, device=device),
            }
            self._dev[key] = t
        return t


_PLANS: Dict[Tuple, Plan] = {}


def plan_for(layout: SegmentLayout, rank: int) -> Plan:
    if not 1 <= rank <= 16:
        raise ValueError("PowerSGD rank must be in [1, 16] (register-resident rows of the tall-skinny kernels / Gram bound)")
    key = (layout.shapes, rank)
    p = _PLANS.get(key)
    if p is not None:
        return p
    mats, vecs = [], []
    po = qo = vo = 0
    for (i, o, n), shape in zip(layout.segments(), layout.shapes):
        if len(shape) >= 2 and n > 0:
            rows = shape[0]
            cols = n // rows
            r = min(rows, cols, rank)
            mats.append((o, rows, cols, r, po, qo))
            po += rows * r
            qo += cols * r
        elif n > 0:
            vecs.append((o, n, vo))
            vo += n
    p = Plan(rank, mats, vecs, po, qo, vo)
    _PLANS[key] = p
    return p


def randn_shared(n: int, seed: int, device, step: Optional[torch.Tensor] = None,
                 zero: Optional[torch.Tensor] = None) -> torch.Tensor:
    """N(0,1) vector identical on every rank for the same seed (and device ``step`` counter,
    mixed in by the kernel when given).  ``zero``: a buffer cleared by the same launch (the P
    that the following :func:`mq` accumulates into: ``mq(..., zeroed=True)``)."""
    if _native.use_native(torch.empty(0, device=device)):
        out = torch.empty(n, dtype=torch.float32, device=device)
        sd = seed & 0xFFFFFFFFFFFFFFFF
        _native.lib().philox_normal(out, sd - (1 << 64) if sd >= (1 << 63) else sd, step, zero)
        return out
    if zero is not None:
        zero.zero_()
    g = torch.Generator(device=device)
    g.manual_seed(seed & 0x7FFFFFFFFFFFFFFF)
    return torch.randn(n, generator=g, device=device)


def _views(buf, plan, which):
    out = []
    for (xo, n, m, r, po, qo) in plan.mats:
        if which == "p":
            out.append(buf[po:po + n * r].view(n, r))
        else:
            out.append(buf[qo:qo + m * r].view(m, r))
    return out


def orthogonalize(buf: torch.Tensor, plan: Plan, which: str, zero: Optional[torch.Tensor] = None) -> None:
    """In-place Gram-Schmidt of the columns of every P_i (or Q_i) -- reference
    dist/compressor/powersgd.py:7-18.  Zero columns stay zero instead of becoming NaN, and a
    column that is numerically dependent on the previous ones (residual below 1e-5 of its norm:
    a rank-deficient P) becomes zero instead of normalised rounding noise (the reference's
    ``col / (norm + 1e-8)`` turns it into an arbitrary non-orthogonal direction).
    ``zero``: a buffer cleared by the same launch (the Q arena the following :func:`mtp` calls
    accumulate into: ``mtp(..., zeroed=True)``)."""
    if zero is not None and not _native.use_native(buf):
        zero.zero_()
    if _native.use_native(buf):
        # Gram-matrix MGS on MFMA, two passes (CholQR2): csrc/kernels/powersgd.hip
        t = plan.tables(buf.device)
        # P = M Q can be ill-conditioned (near-low-rank gradients): CholQR2; the Gaussian Q
        # (condition number ~1) needs one pass
        _native.lib().gram_orthonormalize(buf, t["mat"], 0 if which == "p" else 1, plan.n_mat, t["gt_" + which],
                                          t["gtb_" + which], 2 if which == "p" else 1, plan.rank, zero)
        return
    for a in _views(buf, plan, which):
        r = a.shape[1]
        n0 = torch.sum(a.double() * a.double(), dim=0)  # original squared column norms
        for i in range(r):
            col = a[:, i:i + 1]
            nn = torch.sum(col.double() * col.double())
            # numerically dependent (residual < 1e-5 of the original norm) or zero -> zero column
            # (as the native Gram MGS; normalised cancellation noise would add a spurious direction)
            if nn <= 1e-10 * n0[i] or nn <= 0:
                col.zero_()
            else:
                col /= torch.sqrt(nn).float()
            if i + 1 < r:
                rest = a[:, i + 1:]
                rest -= torch.sum(col * rest, dim=0) * col


def mq(x: torch.Tensor, q: torch.Tensor, plan: Plan, comp_r: Optional[torch.Tensor] = None, beta: float = 1.0,
       gamma: float = 1.0, xout: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
       lazy: Optional[Tuple[torch.Tensor, torch.Tensor, float]] = None, zeroed: bool = False,
       bump: Optional[torch.Tensor] = None, vec: Optional[torch.Tensor] = None) -> torch.Tensor:
    """P_i = M_i Q_i for every matrix (flat P buffer; ``out``: a caller-owned [p_total] view,
    e.g. this bucket's slice of the step-level P arena).

    With ``xout``: M = beta*comp_r + gamma*x (or M = x without ``comp_r``) is also stored into
    ``xout`` for the matrix segments -- the error-feedback compensate fused into this pass.
    ``lazy = (P', Q', s)``: ``comp_r`` holds the previous step's M and the residual is
    comp_r - s P' Q'^T (the previous step's final P and summed Q; the deferred residual update,
    formed here with ``pqt``'s float ops instead of written by it and read back).
    ``zeroed``: ``out`` was already cleared (by :func:`randn_shared`'s launch).  ``bump``: a device
    step counter advanced by this launch (native only).  ``vec`` [v_total]: receives the bucket's
    1-D segments, packed (:func:`gather_vectors`, in the same launch)."""
    p = out if out is not None else torch.empty(plan.p_total, dtype=torch.float32, device=x.device)
    if lazy is not None and comp_r is None:
        raise ValueError("a deferred residual needs comp_r (the previous M)")
    if _native.use_native(x):
        t = plan.tables(x.device)
        lp, lq, ls = lazy if lazy is not None else (None, None, 0.0)
        _native.lib().powersgd_mq(x, q, p, t["mat"], t["tiles0"], 0, comp_r, beta, gamma, xout, plan.rank,
                                  lazy_p=lp, lazy_q=lq, lazy_scale=float(ls), zeroed=bool(zeroed) and out is not None,
                                  bump=bump, vec=vec if plan.v_total else None,
                                  vec_idx=t["vec_idx"] if vec is not None and plan.v_total else None)
        return p
    if bump is not None:
        bump.add_(1)
    if vec is not None:
        vec.copy_(gather_vectors(x, plan))
    for (xo, n, m, r, po, qo) in plan.mats:
        mx = x[xo:xo + n * m]
        if xout is not None:
            cr = comp_r[xo:xo + n * m] if comp_r is not None else None
            if lazy is not None:
                lp, lq, ls = lazy
                o = torch.mm(lp[po:po + n * r].view(n, r), lq[qo:qo + m * r].view(m, r).t()).view(-1)
                cr = cr - (o * ls if ls != 1.0 else o)
            v = beta * cr + gamma * mx if cr is not None else mx
            xout[xo:xo + n * m].copy_(v)
            mx = xout[xo:xo + n * m]
        torch.mm(mx.view(n, m), q[qo:qo + m * r].view(m, r), out=p[po:po + n * r].view(n, r))
    return p


def mtp(x: torch.Tensor, p: torch.Tensor, plan: Plan, out: Optional[torch.Tensor] = None,
        zeroed: bool = False) -> torch.Tensor:
    """Q_i = M_i^T P_i for every matrix (flat Q buffer, or ``out``; ``zeroed``: ``out`` was
    already cleared, by :func:`orthogonalize`'s launch)."""
    q = out if out is not None else torch.empty(plan.q_total, dtype=torch.float32, device=x.device)
    if _native.use_native(x):
        t = plan.tables(x.device)
        _native.lib().powersgd_mq(x, p, q, t["mat"], t["tiles1"], 1, None, 1.0, 1.0, None, plan.rank,
                                  zeroed=bool(zeroed) and out is not None)
        return q
    for (xo, n, m, r, po, qo) in plan.mats:
        torch.mm(x[xo:xo + n * m].view(n, m).t(), p[po:po + n * r].view(n, r), out=q[qo:qo + m * r].view(m, r))
    return q


def mtp_gram(x: torch.Tensor, p: torch.Tensor, plan: Plan, out: torch.Tensor, T: torch.Tensor,
             passes: int = 2) -> None:
    """Native, rank <= 4: ``out`` (cleared beforehand) += M_i^T P_i with P_i as it is (NOT
    orthonormalised), and in the same launch T [n_mat * 16] with P_i T_i orthonormal (CholQR2 in
    the Gram metric, :func:`orthogonalize`'s numerics).  Consumers apply T: the orthonormal factor
    is P T and the PowerSGD Q is (M^T P) T = M^T (P T) (:func:`pqt` ``T=``)."""
    t = plan.tables(x.device)
    _native.lib().powersgd_mtp_gram(x, p, out, t["mat"], t["tiles1"], plan.n_mat, T, int(passes), plan.rank)


def pqt(p: torch.Tensor, q: torch.Tensor, plan: Plan, out: Optional[torch.Tensor], resid: Optional[torch.Tensor] = None,
        scale: float = 1.0, save: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
        vec: Optional[torch.Tensor] = None, vec_scale: float = 1.0, T: Optional[torch.Tensor] = None) -> None:
    """out[matrix i] = scale * P_i Q_i^T (vector segments untouched); with ``resid`` (holding x)
    also resid[matrix i] -= out in the same pass (PowerSGD residual update).  ``scale`` = 1/W
    folds the average of the summed Q into this pass (no separate division kernel).
    ``out=None``: only the residual update (materialising a deferred residual).
    ``save = (P', Q')``: copies of ``p`` and ``q`` stored by the same launch.  ``vec``: the
    packed 1-D segments, scattered into ``out`` times ``vec_scale`` (:func:`scatter_vectors`).
    ``T`` [n_mat * 16] (from :func:`mtp_gram`): ``p`` / ``q`` are taken as P T / Q T (the saved
    copies too)."""
    ref = out if out is not None else resid
    if vec is not None and out is None:
        raise ValueError("pqt: the 1-D segments need out")
    if _native.use_native(ref):
        t = plan.tables(ref.device)
        sp, sq = save if save is not None else (None, None)
        fv = vec is not None and plan.v_total > 0
        _native.lib().powersgd_pqt(p, q, out, t["mat"], t["tilesp"], resid, plan.rank, float(scale), save_p=sp,
                                   save_q=sq, vec=vec.float().contiguous() if fv else None,
                                   vec_idx=t["vec_idx"] if fv else None, vec_scale=float(vec_scale), T=T)
        return
    if T is not None:
        p, q = p.clone(), q.clone()
        for i, (xo, n, m, r, po, qo) in enumerate(plan.mats):
            ti = T[16 * i:16 * i + 16].view(4, 4)[:r, :r]
            p[po:po + n * r] = (p[po:po + n * r].view(n, r) @ ti).reshape(-1)
            q[qo:qo + m * r] = (q[qo:qo + m * r].view(m, r) @ ti).reshape(-1)
    if save is not None:
        save[0].copy_(p)
        save[1].copy_(q)
    if vec is not None:
        scatter_vectors(vec, plan, out, vec_scale)
    for (xo, n, m, r, po, qo) in plan.mats:
        o = torch.mm(p[po:po + n * r].view(n, r), q[qo:qo + m * r].view(m, r).t())
        if scale != 1.0:
            o.mul_(scale)
        if out is not None:
            out[xo:xo + n * m].view(n, m).copy_(o)
        if resid is not None:
            resid[xo:xo + n * m].view(n, m).sub_(o)


def gather_vectors(x: torch.Tensor, plan: Plan) -> torch.Tensor:
    """The 1-D segments of the bucket, packed (one gather kernel on the GPU)."""
    if x.is_cuda:
        return x.index_select(0, plan.tables(x.device)["vec_idx"])
    v = torch.empty(plan.v_total, dtype=torch.float32, device=x.device)
    for (xo, n, vo) in plan.vecs:
        v[vo:vo + n].copy_(x[xo:xo + n])
    return v


def scatter_vectors(v: torch.Tensor, plan: Plan, out: torch.Tensor, scale: float) -> None:
    if out.is_cuda and plan.v_total:
        out.index_copy_(0, plan.tables(out.device)["vec_idx"], v * scale if scale != 1.0 else v)
        return
    for (xo, n, vo) in plan.vecs:
        if scale != 1.0:
            torch.mul(v[vo:vo + n], scale, out=out[xo:xo + n])
        else:
            out[xo:xo + n].copy_(v[vo:vo + n])
