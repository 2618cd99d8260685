"""BatchNorm(+ReLU) -> convolution with the BN apply inside the convolution's GEMM.

In a ResNet bottleneck the outputs of bn1 and bn2 feed exactly one convolution each.  Written
the obvious way every such pair costs an apply pass (read x, write y = act(scale x + shift)),
the consumer conv reading y back, and in backward a BN reduction pass over (dy, x).  Here:

* forward: the producer conv's GEMM emits the BN statistics in its epilogue (ops/conv.py), a
  tiny fold turns them into (mean, invstd, scale, shift) and updates the running statistics,
  and the CONSUMER conv's GEMM applies ``act(scale x + shift)`` to its activation operand as it
  loads it (csrc/kernels/gemm_f32.hip BnApplyPro; the image's zero padding stays zero): y is
  never written to memory;
* backward: the consumer's data-grad GEMM (w.r.t. y) reduces [sum dz | sum dz (x - mean)] in its
  epilogue with the ReLU test recomputed from x (BnBwdEpi), the BN's dx pass runs from those
  partials, and the consumer's weight-grad GEMM recomputes y from x in its operand loader.

Per fused pair: one apply pass, one reduction pass, the y write and the mask write are gone.
Every direction runs on the f32 MFMA GEMM (exact fp32, no xf32); the 3x3 data grad exists for
stride 1, so a strided 3x3 consumer keeps the materialised BN output.  Opt-in
(``GRACE_BN_PROLOGUE=1``): measured slower than the unfused, per-direction autotuned path on
the fp32 headline (see ``_ON``).  Reference for the layer structure:
torchvision ResNet v1.5 bottleneck, as the reference harness trains it
(/root/reference/examples/torch/pytorch_synthetic_benchmark.py:86).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import _native
from . import wgrad as _wg
from .bnact import BatchNormAct2d, _fusable, bn_act

# GRACE_BN_PROLOGUE: 0 = off (default); 1 = bn1 -> conv2 and bn2 -> conv3 fused, measured slower
# on the fp32 ResNet-50 headline (2072 vs 2722 img/s, profiles/r4_bn_fusion_ab.txt: every
# direction of the fused convolutions then runs on the f32 MFMA GEMM, which trails MIOpen's 3x3
# solvers by more than the removed BN passes save); 2 = bn2 -> conv3 only (the 1x1 conv3, where
# the MFMA GEMM is competitive; conv2 keeps its autotuned backend and bn2 a statistics-only pass)
_MODE = int(os.environ.get("GRACE_BN_PROLOGUE", "0") or 0)
_ON = _MODE != 0
_TARGETS = os.environ.get("GRACE_BN_GRAD_TARGET", "1") == "1"


def set_enabled(on, mode: Optional[int] = None) -> None:
    """on: the fused bottleneck path (mode 1 unless ``mode`` is given: 1 full, 2 conv3 only)."""
    global _ON, _MODE
    _ON = bool(on)
    _MODE = (mode if mode is not None else 1) if _ON else 0


def _cl(t: torch.Tensor) -> bool:
    return t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last) and t.data_ptr() % 16 == 0


def bn_fold(bn: BatchNormAct2d, part: torch.Tensor, tiles: int, m: int) -> torch.Tensor:
    """The BN's statistics from GEMM-epilogue partials: save [6C] = (mean, invstd, scale, shift,
    0, 0); running statistics and num_batches_tracked updated as nn.BatchNorm2d does."""
    track = bn.training and bn.track_running_stats
    with torch.no_grad():
        return _native.lib().bn_fold_partials(part, int(tiles), int(m), bn.num_features, bn.weight, bn.bias,
                                              bn.running_mean if track else None, bn.running_var if track else None,
                                              bn.num_batches_tracked if track else None,
                                              float(bn.momentum if bn.momentum is not None else 0.0), float(bn.eps))


class _BnActConvFn(torch.autograd.Function):
    """conv(act(bn(x))) with bn's statistics final in ``save``: the BN apply in the GEMM's
    operand loader; optionally the NEXT BN's statistics from the epilogue (second output)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, save, weight, relu, ksize, want_stats):
        nb, cin, h, w = x.shape
        cout = weight.shape[0]
        m = nb * h * w
        C = _native.lib()
        y = torch.empty((nb, cout, h, w), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
        part = torch.empty(((m + 63) // 64) * 2 * cout, device=x.device, dtype=torch.float32) if want_stats else None
        if ksize == 1:
            wt = weight.reshape(cout, cin)
            t = C.gemm_f32(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 1, 0, part,
                           x_save=save, x_relu=bool(relu), x_op=1)
        else:
            t = C.conv3x3_f32(0, x, weight, y, 1, 1, 0, part, 3, x_save=save, x_relu=bool(relu))
        ctx.save_for_backward(x, gamma, save, weight)
        ctx.conf = (bool(relu), int(ksize))
        ctx.bn_params = (gamma, beta)
        ctx.weight = weight
        if part is None:
            return y
        part._grace_tiles = t
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart=None):
        if dy is None:
            return (None,) * 8
        x, gamma, save, weight = ctx.saved_tensors
        relu, ksize = ctx.conf
        nb, cin, h, w = x.shape
        cout = weight.shape[0]
        m = nb * h * w
        C = _native.lib()
        dy = dy.contiguous(memory_format=torch.channels_last)
        wt = weight.reshape(cout, cin) if ksize == 1 else None
        dx = dg = db = dw = None
        want_x = ctx.needs_input_grad[0]
        want_bn = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        if want_x or want_bn:
            # d(act(bn(x))) on the GEMM, with the BN backward's reduction in its epilogue
            da = torch.empty_like(x, memory_format=torch.channels_last)
            part = torch.empty(((m + 63) // 64) * 2 * cin, device=x.device, dtype=torch.float32)
            if ksize == 1:
                t = C.gemm_f32(dy, True, cout, wt, False, cin, da, cin, m, cin, cout, 1, 0, part, x, None, save, relu)
            else:
                t = C.conv3x3_f32(1, dy, weight, da, 1, 1, 0, part, 3, x, None, save, relu)
            g, b = ctx.bn_params
            tw = _wg.grad_target(g) if (_TARGETS and want_bn) else None
            tb = _wg.grad_target(b) if (_TARGETS and want_bn) else None
            dx, dg, db = C.bn_act_bwd_partials(da, x, None, gamma, save, part, t, relu, want_bn, tw, tb)
            if want_bn:
                dg, db = _wg.into_target(dg, tw), _wg.into_target(db, tb)
        if ctx.needs_input_grad[4]:
            f = _wg.fork(dy, ctx.weight)
            with f as side:
                tgt = _wg.grad_target(ctx.weight)
                if ksize == 1:
                    from .conv import _as_param_layout, _splits

                    o = tgt.reshape(cout, cin) if tgt is not None else \
                        torch.empty((cout, cin), device=x.device, dtype=torch.float32)
                    C.gemm_f32(dy, False, cout, x, False, cin, o, cin, cout, cin, m, _splits(cout, cin, m), 0,
                               x_save=save, x_relu=relu, x_op=2)
                    d = _wg.into_target(_as_param_layout(o, ctx.weight), tgt)
                else:
                    o = tgt if (tgt is not None and _cl(tgt)) else \
                        torch.empty(weight.shape, device=x.device, dtype=torch.float32,
                                    memory_format=torch.channels_last)
                    C.conv3x3_f32(2, x, dy, o, 1, 0, 0, None, 3, x_save=save, x_relu=relu)
                    d = _wg.into_target(o, tgt)
                if side:
                    s = torch.cuda.current_stream(dy.device)
                    _wg.tag(dy, s)
                    _wg.tag(x, s)
                    _wg.tag(save, s)
                    _wg.tag(d, f.main)
            dw = d
        return (dx if want_x else None, dg if ctx.needs_input_grad[1] else None,
                db if ctx.needs_input_grad[2] else None, None, dw, None, None, None)


def _bn_ok(bn, c: int) -> bool:
    """A training-mode fused BN over c channels whose statistics can come from a GEMM epilogue."""
    return (isinstance(bn, BatchNormAct2d) and bn.training and bn.track_running_stats and bn.momentum is not None
            and bn.num_features == c and c % 8 == 0 and c <= 2048 and (c <= 256 or c % 256 == 0))


def bottleneck_main(blk, xm: torch.Tensor, idt: torch.Tensor):
    """The bottleneck's main path conv1 -> bn1 -> conv2 -> bn2 -> conv3 -> bn3(+idt, dual) with
    the bn1 / bn2 applies inside conv2 / conv3 (bn1 materialised when conv2 is strided).
    None when the fused path does not apply (decided before anything runs: the caller then
    runs the plain path)."""
    from .conv import Conv1x1F32, _Conv1x1StatsFn, _Conv3x3StatsFn, fast_ok

    c1, b1, c2, b2, c3, b3 = blk.conv1, blk.bn1, blk.conv2, blk.bn2, blk.conv3, blk.bn3
    if not (_ON and xm.is_cuda and xm.dtype == torch.float32 and torch.is_grad_enabled()
            and not torch.is_autocast_enabled() and _native.native_on(xm.device)):
        return None
    if not (isinstance(c1, Conv1x1F32) and isinstance(c3, Conv1x1F32) and isinstance(c2, _wg.Conv2dSplitGrad)
            and fast_ok(xm, c1, force=True)):
        return None
    w1, w2 = c1.out_channels, c2.out_channels
    if not (_bn_ok(b1, w1) and _bn_ok(b2, w2) and c2.in_channels == w1 and c3.in_channels == w2):
        return None
    # conv2 (3x3, on the implicit GEMM) and conv3 (1x1) on their channels_last fp32 inputs
    from . import conv as _conv

    nb, _, h, w = xm.shape
    s = c2.stride[0]
    ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
    if not (_conv._C3_ON and c2.kernel_size == (3, 3) and c2.padding == (1, 1) and c2.dilation == (1, 1)
            and c2.groups == 1 and c2.bias is None and c2.stride in ((1, 1), (2, 2)) and c2.padding_mode == "zeros"
            and w1 % 32 == 0 and w2 % 32 == 0 and _cl(c2.weight) and nb * h * w < (1 << 24)):
        return None
    if (nb * ho * wo) % 4 or c3.out_channels % 4:
        return None
    if _MODE == 2:
        return _conv3_only(blk, xm, idt)
    # --- run
    y1, p1 = _Conv1x1StatsFn.apply(xm, c1.weight, 0)
    m1 = nb * h * w
    if s == 1:
        s1 = bn_fold(b1, p1, p1._grace_tiles, m1)
        y2, p2 = _BnActConvFn.apply(y1, b1.weight, b1.bias, s1, c2.weight, bool(b1.relu), 3, True)
    else:  # strided 3x3: no implicit-GEMM data grad -> bn1's output is materialised
        a1 = bn_act(y1, b1, None, b1.relu, False, partials=p1, tiles=p1._grace_tiles)
        y2, p2 = _Conv3x3StatsFn.apply(a1, c2.weight, s, 0)
    s2 = bn_fold(b2, p2, p2._grace_tiles, nb * ho * wo)
    y3, p3 = _BnActConvFn.apply(y2, b2.weight, b2.bias, s2, c3.weight, bool(b2.relu), 1, True)
    return bn_act(y3, b3, idt, b3.relu, True, partials=p3, tiles=p3._grace_tiles)


def bn_stats(bn: BatchNormAct2d, y: torch.Tensor) -> torch.Tensor:
    """The BN's statistics by one pass over its input (no apply): save [6C]; running statistics
    and num_batches_tracked updated as nn.BatchNorm2d does."""
    track = bn.training and bn.track_running_stats
    with torch.no_grad():
        return _native.lib().bn_stats_only(y, bn.weight, bn.bias, bn.running_mean if track else None,
                                           bn.running_var if track else None,
                                           bn.num_batches_tracked if track else None,
                                           float(bn.momentum if bn.momentum is not None else 0.0), float(bn.eps))


def _conv3_only(blk, xm: torch.Tensor, idt: torch.Tensor):
    """Mode 2: conv1 -> bn1 -> conv2 as the plain (autotuned) path; bn2's statistics from conv2's
    epilogue when the autotuner chose it, else a statistics-only pass; bn2's apply inside conv3's
    GEMM and its backward reduction in conv3's data-grad epilogue."""
    from .conv import _Conv3x3StatsFn, _pick_bn, conv3x3_ok, conv_bn_act

    c1, b1, c2, b2, c3, b3 = blk.conv1, blk.bn1, blk.conv2, blk.bn2, blk.conv3, blk.bn3
    y1 = conv_bn_act(c1, b1, xm)
    m2 = None
    if conv3x3_ok(y1, c2):
        choice = _pick_bn(c2, b2, y1, None, b2.relu)
        if choice.startswith("stats_t"):
            y2, p2 = _Conv3x3StatsFn.apply(y1, c2.weight, c2.stride[0], int(choice[7:]))
            m2 = y2.shape[0] * y2.shape[2] * y2.shape[3]
            s2 = bn_fold(b2, p2, p2._grace_tiles, m2)
    if m2 is None:
        y2 = c2(y1)
        if not (_cl(y2) and y2.dtype == torch.float32):  # (MIOpen returned another layout: plain path)
            a2 = bn_act(y2, b2, None, b2.relu)
            return bn_act(c3(a2), b3, idt, b3.relu, True)
        s2 = bn_stats(b2, y2)
    y3, p3 = _BnActConvFn.apply(y2, b2.weight, b2.bias, s2, c3.weight, bool(b2.relu), 1, True)
    return bn_act(y3, b3, idt, b3.relu, True, partials=p3, tiles=p3._grace_tiles)


def basic_main(blk, xm: torch.Tensor, idt: torch.Tensor):
    """A basic block's main path conv1 -> bn1 -> conv2 -> bn2(+idt, dual) with bn1 applied inside
    conv2's implicit GEMM; None when it does not apply (decided before anything runs)."""
    from . import conv as _conv

    c1, b1, c2, b2 = blk.conv1, blk.bn1, blk.conv2, blk.bn2
    if not (_ON and _MODE == 1 and xm.is_cuda and xm.dtype == torch.float32 and torch.is_grad_enabled()
            and not torch.is_autocast_enabled() and _native.native_on(xm.device)):
        return None
    if not (isinstance(c1, _wg.Conv2dSplitGrad) and isinstance(c2, _wg.Conv2dSplitGrad)
            and _conv.conv3x3_ok(xm, c1) and c1.kernel_size == (3, 3)):
        return None
    w1, w2 = c1.out_channels, c2.out_channels
    nb, _, h, w = xm.shape
    s = c1.stride[0]
    ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
    if not (_bn_ok(b1, w1) and _bn_ok(b2, w2) and c2.in_channels == w1 and c2.stride == (1, 1)
            and c2.kernel_size == (3, 3) and c2.padding == (1, 1) and c2.dilation == (1, 1) and c2.groups == 1
            and c2.bias is None and c2.padding_mode == "zeros" and w1 % 32 == 0 and w2 % 32 == 0 and _cl(c2.weight)):
        return None
    y1, p1 = _conv._Conv3x3StatsFn.apply(xm, c1.weight, s, 0)
    s1 = bn_fold(b1, p1, p1._grace_tiles, nb * ho * wo)
    y2, p2 = _BnActConvFn.apply(y1, b1.weight, b1.bias, s1, c2.weight, bool(b1.relu), 3, True)
    return bn_act(y2, b2, idt, b2.relu, True, partials=p2, tiles=p2._grace_tiles)
