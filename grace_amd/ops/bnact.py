"""Fused training-mode BatchNorm (+ residual add) (+ ReLU) -- ``BatchNormAct2d``.

A drop-in ``nn.BatchNorm2d`` subclass (same parameters, buffers and state_dict keys) whose
``forward(x, residual=None)`` computes ``act(bn(x) + residual)``.  On a GPU with bf16 or fp32
channels_last activations (bench.py's fp32 default and its bf16 autocast run) it runs the
four CDNA4 kernels of ``csrc/kernels/bnact.hip`` per layer (statistics with the running-stat /
``num_batches_tracked`` update folded in, apply, backward reduce, backward dx) instead of
~11 MIOpen + elementwise launches; everywhere else (CPU, fp32, eval mode, odd channel counts)
it is exactly ``relu(F.batch_norm(x) + residual)``.  fp32 activations use the two-kernel path
(the single-launch variants keep bf16 rows in registers).

Numerics: statistics and the affine are fp32 (forward: fp64 fixed-order fold of the per-block
partial sums; backward: the blocks' partial sums meet in fp32 atomic totals -- order-dependent
to ~1e-7 relative -- unless GRACE_BN_DETERMINISTIC=1 / GRACE_BN_ATOMIC_CHUNKS=0 select the
fixed-order fp64 tree); for
bf16 the output is rounded to bf16 once (the unfused bf16 path rounds after BN, after the add and after
the ReLU); the ReLU mask is taken from the bf16 output, as ``threshold_backward`` does, and kept as 1 bit per
element for the backward (which then reads dy, x and M*C/8 mask bytes instead of dy, x and y).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native
from . import wgrad as _wg


def _fusable(x: torch.Tensor, bn: nn.BatchNorm2d, residual: Optional[torch.Tensor]) -> bool:
    if not (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and _native.native_on(x.device)):
        return False
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last):
        return False
    c = x.shape[1]
    if c % 8 or c > 2048 or (c > 256 and c % 256) or x.numel() == 0 or x.data_ptr() % 16:
        return False
    if residual is not None and (residual.shape != x.shape or residual.stride() != x.stride()
                                 or residual.dtype != x.dtype or residual.data_ptr() % 16):
        return False
    # running statistics: momentum=None (cumulative average) needs the host-side count
    if bn.track_running_stats and bn.momentum is None:
        return False
    return True


_TARGETS = __import__("os").environ.get("GRACE_BN_GRAD_TARGET", "1") == "1"


def _param_targets(ctx, want_w: bool):
    """The bucket views (GRACE engine / DDP comm hook: ops/wgrad.py grad_target) the BN weight
    and bias gradients are written into by the backward kernel itself -- AccumulateGrad then
    steals an alias of the bucket, and neither the engine's gather nor DDP's reducer copies it.
    (None, None) unless both targets exist (a contiguous fp32 [C] view each)."""
    if not want_w or not _TARGETS:
        return None, None
    w, b = ctx.bn_params
    tw = _wg.grad_target(w) if w is not None else None
    tb = _wg.grad_target(b) if b is not None else None
    ok = all(t is not None and t.is_contiguous() and t.dim() == 1 for t in (tw, tb))
    return (tw, tb) if ok else (None, None)


def _kernel_grad(g: Optional[torch.Tensor], like: torch.Tensor) -> Optional[torch.Tensor]:
    if g is None:
        return None
    if g.stride() != like.stride() or g.data_ptr() % 16:
        g = g.contiguous(memory_format=torch.channels_last)
        if g.data_ptr() % 16 or g.stride() != like.stride():
            g = g.clone(memory_format=torch.channels_last)
    return g


# BN -> conv hand-off: a BN(+ReLU) output consumed by exactly ONE convolution (declared by the
# model, e.g. bn1 -> conv2 and bn2 -> conv3 of a ResNet bottleneck) carries a BNHandoff.  The
# consuming conv's data-grad GEMM (ops/conv.py) then also reduces [sum dz | sum dz (x - mean)] in
# its epilogue (gemm_f32.hip BnBwdEpi) and this BN's backward only folds those partials and runs
# its dx pass -- the reduction pass over (dy, x) disappears.  Used only when the gradient handed
# to the BN backward IS the GEMM's output (same storage, no accumulation in between).
_HANDOFF = __import__("os").environ.get("GRACE_BN_BWD_EPI", "0") == "1"  # measured neutral: opt-in


class BNHandoff:
    __slots__ = ("x", "mask", "save", "part", "tiles", "dz_ptr")

    def __init__(self, x, mask, save):
        self.x, self.mask, self.save = x, mask, save
        self.part, self.tiles, self.dz_ptr = None, 0, 0

    def publish(self, part: torch.Tensor, tiles: int, dz: torch.Tensor) -> None:
        self.part, self.tiles, self.dz_ptr = part, int(tiles), dz.data_ptr()


def handoff_of(x: torch.Tensor) -> Optional[BNHandoff]:
    """The BN hand-off of a conv input (None unless the producing BN declared one)."""
    return getattr(x, "_grace_bn_handoff", None) if _HANDOFF else None


class _BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, nbt, momentum, eps, relu, dual,
                partials=None, tiles=0, handoff=False):
        if partials is not None:  # statistics from the producing conv GEMM's epilogue (ops/conv.py)
            y, save, mask = _native.lib().bn_act_fwd_partials(x, residual, partials, int(tiles), weight, bias,
                                                              running_mean, running_var, nbt, float(momentum),
                                                              float(eps), bool(relu))
        else:
            y, save, mask = _native.lib().bn_act_fwd(x, residual, weight, bias, running_mean, running_var, nbt,
                                                     float(momentum), float(eps), bool(relu))
        ctx.relu = bool(relu)
        ctx.has_res = residual is not None
        ctx.bn_params = (weight, bias)
        # the backward needs only the ReLU mask (1 bit per element), not the bf16 output
        ctx.save_for_backward(x, mask if relu else None, weight, save)
        ctx.handoff = None
        if handoff and not dual and residual is None and x.dtype == torch.float32 and x.shape[1] % 8 == 0:
            ctx.handoff = BNHandoff(x, mask if relu else None, save)
            y._grace_bn_handoff = ctx.handoff
        if dual:
            # two aliases of y for two consumers: autograd then hands their gradients to
            # backward() separately and the kernels sum them (no add kernel)
            ctx.set_materialize_grads(False)
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, dy, dy2=None):
        x, mask, weight, save = ctx.saved_tensors
        if dy is None:
            dy, dy2 = dy2, None
        if dy is None:
            return (None,) * 14
        h = ctx.handoff
        if h is not None and h.part is not None and dy2 is None and dy.data_ptr() == h.dz_ptr \
                and dy.stride() == x.stride() and not ctx.has_res:
            part, tiles = h.part, h.tiles
            h.part = None  # one use per backward
            want_w = weight is not None and ctx.needs_input_grad[2]
            tw, tb = _param_targets(ctx, want_w)
            dx, dw, db = _native.lib().bn_act_bwd_partials(dy, x, mask, weight, save, part, tiles, ctx.relu, want_w,
                                                           tw, tb)
            dw, db = _wg.into_target(dw, tw) if want_w else None, _wg.into_target(db, tb) if want_w else None
            return (dx, None, dw, db if ctx.needs_input_grad[3] else None) + (None,) * 10
        dy = _kernel_grad(dy, x)
        dy2 = _kernel_grad(dy2, x)
        want_w = weight is not None and ctx.needs_input_grad[2]
        # the reduce accumulates into totals the forward zeroed: a second backward through the same
        # forward (retain_graph) takes the deterministic fixed-order tree instead
        again = getattr(ctx, "bwd_done", False)
        ctx.bwd_done = True
        tw, tb = _param_targets(ctx, want_w)
        dx, dres, dw, db = _native.lib().bn_act_bwd(dy, dy2, x, mask, weight, save, ctx.relu,
                                                    ctx.has_res and ctx.needs_input_grad[1], want_w, again, tw, tb)
        dw, db = _wg.into_target(dw, tw) if want_w else None, _wg.into_target(db, tb) if want_w else None
        return (dx, dres if ctx.has_res and ctx.needs_input_grad[1] else None,
                dw, db if ctx.needs_input_grad[3] else None,
                None, None, None, None, None, None, None, None, None, None)


def bn_act(x: torch.Tensor, bn: nn.BatchNorm2d, residual: Optional[torch.Tensor] = None,
           relu: bool = False, dual: bool = False, partials: Optional[torch.Tensor] = None, tiles: int = 0,
           handoff: bool = False):
    """``act(bn(x) + residual)`` with the module's parameters and running statistics.

    ``dual=True`` returns ``(y, y_alias)``: two aliases of the output for two consumers (e.g. a
    ResNet block output feeding the next block's conv and its shortcut).  Their gradients reach
    the fused backward separately and are summed inside its kernels instead of by autograd's
    add kernel (one full read+write pass of the activation saved per block).
    ``handoff=True``: the caller guarantees ONE convolution consumes the output (BNHandoff)."""
    training = bn.training or not bn.track_running_stats
    if training and _fusable(x, bn, residual):
        track = bn.training and bn.track_running_stats
        return _BNActFn.apply(x, residual, bn.weight, bn.bias,
                              bn.running_mean if track else None, bn.running_var if track else None,
                              bn.num_batches_tracked if track else None,
                              bn.momentum if bn.momentum is not None else 0.0, bn.eps, relu, bool(dual),
                              partials, tiles, bool(handoff and _HANDOFF))
    y = nn.BatchNorm2d.forward(bn, x)
    if residual is not None:
        y = y + residual
    y = F.relu(y) if relu else y
    return (y, y) if dual else y


class BatchNormAct2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` with an optional fused residual add and ReLU: ``forward(x, residual=None)``."""

    def __init__(self, num_features: int, relu: bool = False, **kw):
        super().__init__(num_features, **kw)
        self.relu = relu

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, dual: bool = False):
        return bn_act(x, self, residual, self.relu, dual)

    def extra_repr(self) -> str:
        return super().extra_repr() + (", relu=True" if self.relu else "")


class _BNActPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, momentum, eps, k, s, pad, dual=False):
        y, save, code = _native.lib().bn_act_pool_fwd(x, weight, bias, running_mean, running_var, nbt,
                                                      float(momentum), float(eps), k, s, pad)
        ctx.geom = (k, s, pad)
        ctx.bn_params = (weight, bias)
        ctx.save_for_backward(x, code, weight, save)
        if dual:
            # two aliases for the two consumers (the first block's main path and shortcut): their
            # gradients arrive separately and the max-pool backward sums them (no add kernel:
            # 28 us per ResNet-50 step)
            ctx.set_materialize_grads(False)
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, dp, dp2=None):
        x, code, weight, save = ctx.saved_tensors
        k, s, pad = ctx.geom
        if dp is None:
            dp, dp2 = dp2, None
        if dp is None:
            return (None,) * 12

        def cl(t):
            if not t.is_contiguous(memory_format=torch.channels_last) or t.data_ptr() % 16:
                t = t.contiguous(memory_format=torch.channels_last)
                if t.data_ptr() % 16:
                    t = t.clone(memory_format=torch.channels_last)
            return t

        dp = cl(dp)
        dp2 = cl(dp2) if dp2 is not None else None
        C = _native.lib()
        dy = C.maxpool_bwd(dp, code, x.shape[2], x.shape[3], k, s, pad, dy2=dp2)  # gradient of relu(bn(x))
        want_w = weight is not None and ctx.needs_input_grad[1]
        # mask None: the ReLU mask is recomputed from x and save's scale / shift
        again = getattr(ctx, "bwd_done", False)
        ctx.bwd_done = True
        tw, tb = _param_targets(ctx, want_w)
        dx, _, dw, db = C.bn_act_bwd(dy, None, x, None, weight, save, True, False, want_w, again, tw, tb)
        dw, db = _wg.into_target(dw, tw) if want_w else None, _wg.into_target(db, tb) if want_w else None
        return (dx, dw, db if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, None, None, None, None)


def bn_relu_maxpool(x: torch.Tensor, bn: "BatchNormAct2d", pool: nn.MaxPool2d, dual: bool = False):
    """``pool(relu(bn(x)))`` -- the ResNet stem -- as stats + ONE normalise/ReLU/pool pass forward
    (the 103 MB BN output and its ReLU mask are never written; csrc/kernels/bnact.hip
    bn_pool_apply_kernel); backward = the gather max-pool backward + the BN backward with the
    ReLU mask recomputed from x.  Other configurations run ``pool(bn(x))`` through the modules.
    ``dual``: the fused path returns two aliases of the output for two consumers (their gradients
    are summed by the max-pool backward); the fallback returns the plain tensor."""
    from .pool import MaxPool2dNHWC

    training = bn.training or not bn.track_running_stats
    if (training and bn.relu and isinstance(pool, MaxPool2dNHWC) and pool._native_ok(x)
            and _fusable(x, bn, None)):
        k = pool.kernel_size if isinstance(pool.kernel_size, int) else pool.kernel_size[0]
        st = pool.stride if isinstance(pool.stride, int) else (pool.stride or pool.kernel_size)[0]
        pd = pool.padding if isinstance(pool.padding, int) else pool.padding[0]
        track = bn.training and bn.track_running_stats
        return _BNActPoolFn.apply(x, bn.weight, bn.bias, bn.running_mean if track else None,
                                  bn.running_var if track else None, bn.num_batches_tracked if track else None,
                                  bn.momentum if bn.momentum is not None else 0.0, bn.eps, k, st, pd, bool(dual))
    return pool(bn(x))
