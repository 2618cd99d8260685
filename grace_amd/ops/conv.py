"""fp32 1x1 convolutions of channels_last activations on the hand-written f32 MFMA GEMM.

A 1x1 stride-1 convolution over a channels_last activation is a plain GEMM over its
[M = N*H*W, C] view (no im2col), so all three of its products run on
``csrc/kernels/gemm_f32.hip`` (``v_mfma_f32_32x32x2_f32``, exact fp32):

    forward      Y[M, Cout]    = X[M, Cin] . W[Cout, Cin]^T
    data grad    dX[M, Cin]    = dY[M, Cout] . W[Cout, Cin]
    weight grad  dW[Cout, Cin] = dY^T . X           (split-K over M, f32 atomics)

``Conv1x1F32`` is a drop-in ``nn.Conv2d`` subclass (same parameters / state_dict) used by the
ResNet bottlenecks; it falls back to ``F.conv2d`` whenever the fast path does not apply (CPU,
bf16/autocast, non-channels_last input, odd channel counts, stride/padding/groups/bias).

Per-direction autotuned dispatch (``GRACE_CONV_AUTO=1``, the default for fp32 channels_last):
every 1x1 stride-1 layer times, once per (shape, direction) on the device, three backends
-- MIOpen (``F.conv2d`` / ``aten.convolution_backward``; its time INCLUDES the zero-fill
``SubTensorOpWithScalar1d`` kernels its implicit-GEMM solvers launch before every call), the
hipBLASLt GEMM on the [M, C] views (``torch.mm``, no im2col, no fill) and the hand-written f32
MFMA GEMM -- and keeps the fastest for that direction.  Decisions are taken in eager steps
(never while a stream is being captured; a captured graph replays them) and are listed by
``autotune_table()``.  ``GRACE_CONV_MFMA=1`` forces the MFMA GEMM for all three directions
(measured per layer on ResNet-50 b32 within ~10 % of MIOpen's solvers,
profiles/r2_conv_fp32_mfma_vs_miopen.txt).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native
from . import bnact as _bn
from . import wgrad as _wg

_TARGET_BLOCKS = 512  # >> 256 CUs


def _splits(m: int, n: int, k: int) -> int:
    tm = (m + 127) // 128 if m > 64 else 1
    tn = (n + 127) // 128 if n > 64 or m <= 64 else 1
    tiles = tm * tn
    return max(1, min(math.ceil(_TARGET_BLOCKS / tiles), k // 256))


def gemm(a, a_kc, lda, b, b_kc, ldb, c, ldc, m, n, k, splits=1, tile=0):
    """C[m, n] = sum_k A(m, k) B(n, k) (see csrc/kernels/gemm_f32.hip); splits=0: split-K chosen by
    the launcher when the output has too few tiles to fill the chip (needs a dense C); tile:
    0 = launcher's rule, 1 = 128x128, 2 = 128x64, 3 = 64x128, 4 = 64x64 (5-7: aliases of 2-4)."""
    _native.lib().gemm_f32(a, a_kc, lda, b, b_kc, ldb, c, ldc, m, n, k, splits, tile)


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        nb, cin, h, w = x.shape
        cout = weight.shape[0]
        m = nb * h * w
        wt = weight.reshape(cout, cin)
        if not wt.is_contiguous():
            wt = wt.contiguous()
        y = torch.empty((nb, cout, h, w), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
        gemm(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 0)
        ctx.save_for_backward(x, wt)
        ctx.wshape = weight.shape
        ctx.weight = weight
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        nb, cin, h, w = x.shape
        cout = wt.shape[0]
        m = nb * h * w
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            gemm(dy, True, cout, wt, False, cin, dx, cin, m, cin, cout, 0)
        if ctx.needs_input_grad[1]:
            f = _wg.fork(dy, ctx.weight)
            with f as side:
                dw = torch.empty((cout, cin), device=x.device, dtype=torch.float32)
                gemm(dy, False, cout, x, False, cin, dw, cin, cout, cin, m, _splits(cout, cin, m))
                dw = _as_param_layout(dw, ctx.weight)
                if side:
                    s = torch.cuda.current_stream(dy.device)
                    _wg.tag(dy, s)
                    _wg.tag(x, s)
                    _wg.tag(dw, f.main)
        return dx, dw


_ENABLED = os.environ.get("GRACE_CONV_MFMA", "0") == "1"
_AUTO = os.environ.get("GRACE_CONV_AUTO", "1") == "1"

# (direction, M, Cin, Cout) -> backend name; and the measured times (ms) per backend
_CHOICE = {}
_TIMES = {}
BACKENDS = ("miopen", "hipblaslt", "mfma", "mfma_t1", "mfma_t2", "mfma_t3", "mfma_t4")


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


def set_autotune(on: bool) -> None:
    global _AUTO
    _AUTO = bool(on)


def autotune_table():
    """[(direction, M, Cin, Cout, chosen, {backend: ms})] of every tuned layer direction."""
    return [(k[0], k[1], k[2], k[3], v, dict(_TIMES.get(k, {}))) for k, v in sorted(_CHOICE.items())]


def _as_param_layout(dw2d: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """A dense [Cout, Cin] weight gradient viewed with the 1x1 weight's own strides (the memory
    image is the same whatever the strides of the size-1 dims): DDP's reducer compares strides
    literally and would otherwise copy every such gradient into its bucket view."""
    if dw2d.is_contiguous() and weight.dim() == 4 and weight.shape[2] == 1 and weight.shape[3] == 1 \
            and weight.stride(1) == 1 and weight.stride(0) == weight.shape[1]:
        return dw2d.as_strided(weight.shape, weight.stride())
    return dw2d.view(weight.shape)


def _x2d(t: torch.Tensor) -> torch.Tensor:
    """[M, C] view of a channels_last NCHW tensor."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _cl_from_2d(y2d: torch.Tensor, nb: int, h: int, w: int) -> torch.Tensor:
    return y2d.view(nb, h, w, -1).permute(0, 3, 1, 2)


def _run(direction: str, backend: str, x, wt, dy, wshape, out=None):
    """One direction on one backend.  x: [N, Cin, H, W] channels_last; wt: [Cout, Cin]; dy:
    [N, Cout, H, W] channels_last (backward) -- returns y / dx (channels_last) / dw [Cout, Cin].
    ``out`` (wgrad only): a dense [Cout, Cin] destination (the engine's bucket view) the GEMM
    backends write in place."""
    nb, cin, h, w = x.shape
    cout = wt.shape[0]
    m = nb * h * w
    if backend == "miopen":
        w4 = wt.view(wshape)
        if direction == "fwd":
            return F.conv2d(x, w4)
        mask = [direction == "dgrad", direction == "wgrad", False]
        gi, gw, _ = torch.ops.aten.convolution_backward(dy, x, w4, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1,
                                                        mask)
        return gi if direction == "dgrad" else gw.reshape(cout, cin)
    if backend == "hipblaslt":
        if direction == "fwd":
            return _cl_from_2d(torch.mm(_x2d(x), wt.t()), nb, h, w)
        if direction == "dgrad":
            return _cl_from_2d(torch.mm(_x2d(dy), wt), nb, h, w)
        if out is not None:
            return torch.mm(_x2d(dy).t(), _x2d(x), out=out)
        return torch.mm(_x2d(dy).t(), _x2d(x))
    # mfma[_tN]: csrc/kernels/gemm_f32.hip with the launcher's tile rule or a forced tile
    tile = _tile_of(backend)
    if direction == "fwd":
        y = torch.empty((nb, cout, h, w), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
        gemm(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 0, tile)
        return y
    if direction == "dgrad":
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        gemm(dy, True, cout, wt, False, cin, dx, cin, m, cin, cout, 0, tile)
        return dx
    dw = out if out is not None else torch.empty((cout, cin), device=x.device, dtype=torch.float32)
    gemm(dy, False, cout, x, False, cin, dw, cin, cout, cin, m, _splits(cout, cin, m), tile)
    return dw


def _pick(direction: str, x, wt, dy, wshape) -> str:
    if _ENABLED:
        return "mfma"
    nb, cin, h, w = x.shape
    key = (direction, nb * h * w, cin, wt.shape[0])
    c = _CHOICE.get(key)
    if c is not None:
        return c
    if torch.cuda.is_current_stream_capturing():
        return "miopen"  # never time inside a capture
    times = {}
    for be in BACKENDS:
        try:
            times[be] = _time(lambda be=be: _run(direction, be, x, wt, dy, wshape))
        except Exception:  # a backend that rejects the shape is simply not a candidate
            continue
    c = min(times, key=times.get) if times else "miopen"
    _CHOICE[key] = c
    _TIMES[key] = times
    return c


def _tile_of(backend: str) -> int:
    return _mfma_cfg(backend)[0]


def _mfma_cfg(backend: str):
    """(tile, splits) of an "mfma[_tN][_sK]" backend name (tile 0 = the launcher's rule; splits 0 =
    the caller's default)."""
    tile = splits = 0
    for tok in backend.split("_")[1:]:
        if tok.startswith("t"):
            tile = int(tok[1:])
        elif tok.startswith("s"):
            splits = int(tok[1:])
    return tile, splits


def _dgrad_handoff(h, x, w, dy, ksize: int, tile: int = 0):
    """Data grad on the MFMA GEMM with the producing BN's backward reduction in its epilogue
    (ops/bnact.py BNHandoff); None when it does not apply.  ksize 1: w is [Cout, Cin] (plain
    GEMM); 3: the channels_last 3x3 weight (implicit GEMM, stride 1)."""
    if h is None or h.x.shape != x.shape or not h.x.is_contiguous(memory_format=torch.channels_last):
        return None
    nb, cin, hh, ww = x.shape
    m = nb * hh * ww
    dx = torch.empty_like(x, memory_format=torch.channels_last)
    part = torch.empty(((m + 63) // 64) * 2 * cin, device=x.device, dtype=torch.float32)
    C = _native.lib()
    if ksize == 1:
        cout = w.shape[0]
        t = C.gemm_f32(dy, True, cout, w, False, cin, dx, cin, m, cin, cout, 1, tile, part, h.x, h.mask, h.save)
    else:
        t = C.conv3x3_f32(1, dy, w, dx, 1, 1, tile, part, 3, h.x, h.mask, h.save)
    h.publish(part, t, dx)
    return dx


class _Conv1x1AutoFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        cout, cin = weight.shape[0], weight.shape[1]
        wt = weight.reshape(cout, cin)
        if not wt.is_contiguous():
            wt = wt.contiguous()
        y = _run("fwd", _pick("fwd", x, wt, None, weight.shape), x, wt, None, weight.shape)
        ctx.save_for_backward(x, wt)
        ctx.wshape = weight.shape
        ctx.weight = weight
        ctx.bn_h = _bn.handoff_of(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wt = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        f = None
        if ctx.needs_input_grad[1]:
            f = _wg.fork(dy, ctx.weight)

        def wg():
            be = _pick("wgrad", x, wt, dy, ctx.wshape)  # autotuned on the current stream, never on the side one
            # the engine's bucket view, written in place by the GEMM backends (MIOpen's own output
            # would need a copy kernel on the side stream's critical tail: left to the gather)
            tgt = _wg.grad_target(ctx.weight) if (be != "miopen" or _wg.must_alias(ctx.weight)) else None
            with f as side:  # wgrad off the critical path (ops/wgrad.py)
                o2 = tgt.reshape(wt.shape) if tgt is not None else None
                d = _wg.into_target(_as_param_layout(_run("wgrad", be, x, wt, dy, ctx.wshape, out=o2), ctx.weight), tgt)
                if side:
                    s = torch.cuda.current_stream(dy.device)
                    _wg.tag(dy, s)
                    _wg.tag(x, s)
                    _wg.tag(d, f.main)
            return d

        if ctx.needs_input_grad[0]:
            be = _pick("dgrad", x, wt, dy, ctx.wshape)
            # the producing BN's reduction in the epilogue -- only where the MFMA GEMM is already the
            # measured-fastest data grad (forcing it elsewhere measured slower overall)
            dx = _dgrad_handoff(getattr(ctx, "bn_h", None), x, wt, dy, 1, _tile_of(be)) \
                if be.startswith("mfma") else None
            if dx is None:
                dx = _run("dgrad", be, x, wt, dy, ctx.wshape)
        if f is not None:
            dw = wg()
        return dx, dw


class _Conv1x1StatsFn(torch.autograd.Function):
    """Forward on the MFMA GEMM whose epilogue also emits the per-(row tile, channel) sum / sum of
    squares of the output (the following BatchNorm's statistics: its statistics pass over the
    activation disappears); backward = the autotuned dgrad / wgrad of _Conv1x1AutoFn."""

    @staticmethod
    def forward(ctx, x, weight, tile):
        nb, cin, h, w = x.shape
        cout = weight.shape[0]
        m = nb * h * w
        wt = weight.reshape(cout, cin)
        if not wt.is_contiguous():
            wt = wt.contiguous()
        y = torch.empty((nb, cout, h, w), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
        part = torch.empty(((m + 63) // 64) * 2 * cout, device=x.device, dtype=torch.float32)
        part._grace_tiles = _native.lib().gemm_f32(x, True, cin, wt, True, cin, y, cout, m, cout, cin, 1, int(tile),
                                                   part)
        ctx.save_for_backward(x, wt)
        ctx.wshape = weight.shape
        ctx.weight = weight
        ctx.bn_h = _bn.handoff_of(x)
        ctx.mark_non_differentiable(part)
        # the statistics output never gets a gradient: without this autograd would materialise a
        # zero tensor for it in every backward (one fill kernel per layer on the critical path)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart=None):
        if dy is None:  # (not materialised) nothing flowed into the conv output
            x, wt = ctx.saved_tensors
            return None, None, None
        dx, dw = _Conv1x1AutoFn.backward(ctx, dy)
        return dx, dw, None


def _tiles_m(m: int, tile: int) -> int:
    return (m + 127) // 128 if tile in (1, 2) else (m + 63) // 64


# (M, Cin, Cout, relu, residual) -> "unfused" | "stats_t<tile>" ; measured ms per candidate
_BN_CHOICE = {}
_BN_TIMES = {}
_BN_FUSE = os.environ.get("GRACE_CONV_BN_STATS", "1") == "1"


def _time(fn, reps=5, trials=3):
    """ms per call: the best of ``trials`` runs of ``reps`` calls (near-ties between backends
    otherwise flip from run to run)."""
    for _ in range(2):
        fn()
    best = float("inf")
    for _ in range(trials):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    return best


def _pick_bn(conv, bn, x, residual, relu) -> str:
    nb, cin, h, w = x.shape
    k3 = conv.kernel_size == (3, 3) or conv.stride != (1, 1)  # implicit-GEMM conv (3x3 or strided 1x1)
    s = conv.stride[0]
    key = (nb * h * w, cin, conv.out_channels, bool(relu), residual is not None) + ((3, s) if k3 else ())
    c = _BN_CHOICE.get(key)
    if c is not None:
        return c
    if torch.cuda.is_current_stream_capturing():
        return "unfused"
    C = _native.lib()
    cout = conv.out_channels
    wt = conv.weight.detach().reshape(cout, cin).contiguous() if not k3 else None
    w4 = conv.weight.detach()
    rm, rv = torch.zeros(cout, device=x.device), torch.ones(cout, device=x.device)
    nbt = torch.zeros((), dtype=torch.int64, device=x.device)
    g, b = bn.weight.detach(), bn.bias.detach()
    res = residual.detach() if residual is not None else None
    xd = x.detach()
    ho, wo = ((h - 1) // s + 1, (w - 1) // s + 1) if k3 else (h, w)
    m = nb * ho * wo
    times = {}

    def unfused():
        if k3:
            y = _run3("fwd", _pick3("fwd", xd, w4, None, s), xd, w4, None, s)
        else:
            y = _run("fwd", _pick("fwd", xd, wt, None, w4.shape), xd, wt, None, w4.shape)
        C.bn_act_fwd(y, res, g, b, rm, rv, nbt, 0.1, 1e-5, bool(relu))

    times["unfused"] = _time(unfused)
    part = torch.empty(((m + 63) // 64) * 2 * cout, device=x.device)
    for tile in (1, 2, 3, 4):
        def fused(tile=tile):
            y = torch.empty((nb, cout, ho, wo), device=x.device, memory_format=torch.channels_last)
            if k3:
                t = C.conv3x3_f32(0, xd, w4, y, s, 1, tile, part, w4.shape[2])
            else:
                t = C.gemm_f32(xd, True, cin, wt, True, cin, y, cout, m, cout, cin, 1, tile, part)
            C.bn_act_fwd_partials(y, res, part, t, g, b, rm, rv, nbt, 0.1, 1e-5, bool(relu))
        try:
            times[f"stats_t{tile}"] = _time(fused)
        except Exception:
            continue
    c = min(times, key=times.get)
    _BN_CHOICE[key] = c
    _BN_TIMES[key] = times
    return c


def bn_autotune_table():
    """[(M, Cin, Cout, relu, residual, chosen, {candidate: ms})] of the conv -> BN forward pairs."""
    return [k + (v, dict(_BN_TIMES.get(k, {}))) for k, v in sorted(_BN_CHOICE.items())]


def conv_bn_act(conv: nn.Module, bn: nn.Module, x: torch.Tensor, residual=None, dual: bool = False,
                handoff: bool = False):
    """``bn(conv(x), residual, dual)`` for a 1x1 stride-1 ``Conv1x1F32`` or a 3x3 implicit-GEMM
    convolution (``conv3x3_ok``) followed by a fused
    ``BatchNormAct2d``: when the autotuner measured it faster (GEMM + statistics epilogue + fold +
    apply vs the best conv backend + the BN statistics and apply passes, each timed whole), the
    conv runs on the MFMA GEMM that also emits the BN statistics, and the BN skips its
    statistics pass over the activation.  Otherwise exactly ``bn(conv(x), residual, dual=dual)``."""
    from .bnact import BatchNormAct2d, _fusable, bn_act

    relu = getattr(bn, "relu", False)
    bn_ok = _BN_FUSE and bn.training and bn.track_running_stats and bn.momentum is not None
    if (bn_ok and not _ENABLED and isinstance(conv, Conv1x1F32) and fast_ok(x, conv)
            and x.shape[0] * x.shape[2] * x.shape[3] < (1 << 31)):
        choice = _pick_bn(conv, bn, x, residual, relu)
        if choice.startswith("stats_t"):
            tile = int(choice[7:])
            y, part = _Conv1x1StatsFn.apply(x, conv.weight, tile)
            if _fusable(y, bn, residual):
                m = x.shape[0] * x.shape[2] * x.shape[3]
                return bn_act(y, bn, residual, relu, dual, partials=part, tiles=_tiles_m(m, tile), handoff=handoff)
            return bn(y, residual, dual=dual)
    if bn_ok and isinstance(conv, _wg.Conv2dSplitGrad) and conv3x3_ok(x, conv):
        choice = _pick_bn(conv, bn, x, residual, relu)
        if choice.startswith("stats_t"):
            tile = int(choice[7:])
            y, part = _Conv3x3StatsFn.apply(x, conv.weight, conv.stride[0], tile)
            if _fusable(y, bn, residual):
                m = y.shape[0] * y.shape[2] * y.shape[3]
                return bn_act(y, bn, residual, relu, dual, partials=part, tiles=_tiles_m(m, tile), handoff=handoff)
            return bn(y, residual, dual=dual)
    if handoff and isinstance(bn, BatchNormAct2d):
        return bn_act(conv(x), bn, residual, relu, dual, handoff=True)
    return bn(conv(x), residual, dual=dual)


def fast_ok(x: torch.Tensor, conv: nn.Conv2d, force: bool = False) -> bool:
    if not (_ENABLED or _AUTO or force):
        return False
    if not (x.is_cuda and x.dtype == torch.float32 and conv.weight.dtype == torch.float32):
        return False
    if torch.is_autocast_enabled() or not _native.native_on(x.device):
        return False
    if conv.kernel_size != (1, 1) or conv.stride != (1, 1) or conv.padding != (0, 0) or conv.groups != 1 \
            or conv.dilation != (1, 1) or conv.bias is not None:
        return False
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16:
        return False
    cin, cout = conv.in_channels, conv.out_channels
    return cin % 4 == 0 and cout % 4 == 0 and x.shape[0] * x.shape[2] * x.shape[3] % 4 == 0


# ---------------------------------------------------------------- 3x3 convolutions
# The 3x3 / pad 1 convolutions run as implicit GEMMs on the same f32 MFMA kernel (gemm_f32.hip:
# the operand loader gathers the shifted NHWC pixels; no im2col buffer, no zero-fill kernel before
# the forward or the data grad).  Per layer and direction the autotuner times MIOpen (including
# its zero fills) against the implicit GEMM's tile shapes and keeps the fastest.
_C3_CHOICE = {}
_C3_TIMES = {}
C3_BACKENDS = ("miopen", "mfma", "mfma_t1", "mfma_t2", "mfma_t3", "mfma_t4")
# split-K variants for the forward / data grad of the small-M layers (14x14 / 7x7 at batch 32:
# M = N*H*W of 6272 / 1568 leaves most of the 256 CUs idle with whole-K tiles, and a 64x64 tile
# is latency bound -- 32 k per LDS stage is too little MFMA work to cover a global load); every
# split accumulates with f32 atomics into a zeroed output.  Only candidates whose whole-K tiling
# leaves CUs idle are timed (_c3_candidates).
C3_SPLIT_BACKENDS = ("mfma_t1_s2", "mfma_t1_s4", "mfma_t2_s2", "mfma_t2_s4", "mfma_t3_s2", "mfma_t3_s4",
                     "mfma_t4_s2")
_TILE_MN = {1: (128, 128), 2: (128, 64), 3: (64, 128), 4: (64, 64)}


def _c3_candidates(direction: str, m: int, n: int):
    if direction == "wgrad":
        return C3_BACKENDS  # split-K by the launcher's own rule (K = output pixels)
    out = list(C3_BACKENDS)
    for be in C3_SPLIT_BACKENDS:
        t, s = _mfma_cfg(be)
        bm, bn = _TILE_MN[t]
        if -(-m // bm) * -(-n // bn) * s <= 2 * 256 * 2 and -(-m // bm) * -(-n // bn) < 256:
            out.append(be)
    return tuple(out)
_C3_ON = os.environ.get("GRACE_CONV3X3", "1") == "1"


def conv3x3_ok(x: torch.Tensor, conv: nn.Conv2d, bias_ok: bool = False) -> bool:
    """The implicit-GEMM path applies: fp32 channels_last activation and weight, 3x3 / pad 1 /
    stride 1 or 2, no groups / dilation, no bias (unless the caller adds it: ``bias_ok``),
    channels multiples of 32."""
    if not (_C3_ON and (_AUTO or _ENABLED)):
        return False
    w = conv.weight
    if not (x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32):
        return False
    if torch.is_autocast_enabled() or not _native.native_on(x.device):
        return False
    k3 = conv.kernel_size == (3, 3) and conv.padding == (1, 1)
    k1s = conv.kernel_size == (1, 1) and conv.padding == (0, 0) and conv.stride == (2, 2)  # strided 1x1
    if not (k3 or k1s) or conv.dilation != (1, 1) or conv.groups != 1 \
            or (conv.bias is not None and not bias_ok) or conv.stride not in ((1, 1), (2, 2)) \
            or conv.padding_mode != "zeros":
        return False
    if x.dim() != 4 or not x.is_contiguous(memory_format=torch.channels_last) or x.data_ptr() % 16:
        return False
    if not w.is_contiguous(memory_format=torch.channels_last) or w.data_ptr() % 16:
        return False
    return conv.in_channels % 32 == 0 and conv.out_channels % 32 == 0 \
        and x.shape[0] * x.shape[2] * x.shape[3] < (1 << 24)


def _run3(direction: str, backend: str, x, w, dy, stride: int, out=None):
    """One direction of a 3x3 / pad 1 (or strided 1x1 / pad 0) conv on one backend (x, dy, w
    channels_last)."""
    ks = w.shape[2]
    pad = (ks - 1) // 2
    if backend == "miopen":
        if direction == "fwd":
            return F.conv2d(x, w, None, stride, pad)
        mask = [direction == "dgrad", direction == "wgrad", False]
        gi, gw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad], [1, 1], False,
                                                        [0, 0], 1, mask)
        return gi if direction == "dgrad" else gw
    tile, splits = _mfma_cfg(backend)
    splits = max(1, splits)  # forward / data grad: whole-K tiles unless the backend splits K
    C = _native.lib()
    nb, cin, h, wd = x.shape
    cout = w.shape[0]
    if direction == "fwd":
        ho, wo = (h - 1) // stride + 1, (wd - 1) // stride + 1
        y = torch.empty((nb, cout, ho, wo), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
        C.conv3x3_f32(0, x, w, y, stride, splits, tile, None, ks)
        return y
    if direction == "dgrad":
        if stride != 1 or ks != 3:
            raise ValueError("implicit-GEMM data grad: 3x3 stride 1 only")
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        C.conv3x3_f32(1, dy, w, dx, 1, splits, tile)
        return dx
    dw = out if (out is not None and out.is_contiguous(memory_format=torch.channels_last)
                 and out.data_ptr() % 16 == 0) else \
        torch.empty((cout, cin, ks, ks), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
    C.conv3x3_f32(2, x, dy, dw, stride, 0, tile, None, ks)
    return dw


def _pick3(direction: str, x, w, dy, stride: int) -> str:
    nb, cin, h, wd = x.shape
    key = (direction, nb, h, wd, cin, w.shape[0], stride, w.shape[2])
    c = _C3_CHOICE.get(key)
    if c is not None:
        return c
    if direction == "dgrad" and (stride != 1 or w.shape[2] != 3):
        return "miopen"
    if _ENABLED:
        return "mfma"
    if torch.cuda.is_current_stream_capturing():
        return "miopen"  # never time inside a capture
    times = {}
    ho, wo = (h - 1) // stride + 1, (wd - 1) // stride + 1
    m, n = (nb * h * wd, cin) if direction == "dgrad" else (nb * ho * wo, w.shape[0])
    for be in _c3_candidates(direction, m, n):
        try:
            times[be] = _time(lambda be=be: _run3(direction, be, x, w, dy, stride))
        except Exception:  # a backend that rejects the shape is simply not a candidate
            continue
    c = min(times, key=times.get) if times else "miopen"
    _C3_CHOICE[key] = c
    _C3_TIMES[key] = times
    return c


def conv3x3_autotune_table():
    """[(direction, N, H, W, Cin, Cout, stride, ksize, chosen, {backend: ms})] of every tuned direction."""
    return [k + (v, dict(_C3_TIMES.get(k, {}))) for k, v in sorted(_C3_CHOICE.items())]


class _Conv3x3Fn(torch.autograd.Function):
    """3x3 / pad 1 conv: each direction on its autotuned backend; the weight gradient on the
    side stream / deferred / into the engine's bucket view exactly like the 1x1 path."""

    @staticmethod
    def forward(ctx, x, weight, stride):
        y = _run3("fwd", _pick3("fwd", x, weight, None, stride), x, weight, None, stride)
        ctx.save_for_backward(x, weight)
        ctx.stride = stride
        ctx.weight = weight
        ctx.bn_h = _bn.handoff_of(x) if stride == 1 and weight.shape[2] == 3 else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride = ctx.stride
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        f = None
        if ctx.needs_input_grad[1]:
            f = _wg.fork(dy, ctx.weight)

        def wg():
            be = _pick3("wgrad", x, w, dy, stride)  # autotuned on the current stream
            tgt = _wg.grad_target(ctx.weight) if (be != "miopen" or _wg.must_alias(ctx.weight)) else None
            with f as side:
                d = _wg.into_target(_run3("wgrad", be, x, w, dy, stride, out=tgt), tgt)
                if side:
                    s = torch.cuda.current_stream(dy.device)
                    _wg.tag(dy, s)
                    _wg.tag(x, s)
                    _wg.tag(d, f.main)
            return d

        if ctx.needs_input_grad[0]:
            be = _pick3("dgrad", x, w, dy, stride)
            dx = _dgrad_handoff(getattr(ctx, "bn_h", None), x, w, dy, 3, _tile_of(be)) \
                if be.startswith("mfma") and _mfma_cfg(be)[1] <= 1 else None
            if dx is None:
                dx = _run3("dgrad", be, x, w, dy, stride)
        if f is not None:
            dw = wg()
        return dx, dw, None


class _Conv3x3StatsFn(torch.autograd.Function):
    """3x3 forward on the implicit GEMM whose epilogue also emits the following BatchNorm's
    per-(row tile, channel) sum / sum of squares; backward = _Conv3x3Fn's."""

    @staticmethod
    def forward(ctx, x, weight, stride, tile):
        nb, cin, h, w = x.shape
        cout = weight.shape[0]
        ho, wo = (h - 1) // stride + 1, (w - 1) // stride + 1  # 3x3 pad 1 or 1x1 pad 0
        y = torch.empty((nb, cout, ho, wo), device=x.device, dtype=torch.float32, memory_format=torch.channels_last)
        part = torch.empty(((nb * ho * wo + 63) // 64) * 2 * cout, device=x.device, dtype=torch.float32)
        part._grace_tiles = _native.lib().conv3x3_f32(0, x, weight, y, stride, 1, int(tile), part, weight.shape[2])
        ctx.save_for_backward(x, weight)
        ctx.stride = stride
        ctx.weight = weight
        ctx.bn_h = _bn.handoff_of(x) if stride == 1 and weight.shape[2] == 3 else None
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)  # no zero tensor for the statistics' gradient
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart=None):
        if dy is None:
            return None, None, None, None
        dx, dw, _ = _Conv3x3Fn.backward(ctx, dy)
        return dx, dw, None, None


class Conv1x1F32(_wg.Conv2dSplitGrad):
    """``nn.Conv2d(cin, cout, 1, bias=False)`` whose fp32 channels_last path runs on the f32 MFMA GEMM."""

    def __init__(self, cin: int, cout: int, **kw):
        super().__init__(cin, cout, 1, bias=False, **kw)

    def forward(self, x):
        if fast_ok(x, self):
            return (_Conv1x1Fn if _ENABLED else _Conv1x1AutoFn).apply(x, self.weight)
        return super().forward(x)
