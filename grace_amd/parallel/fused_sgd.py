"""``FusedSGD``: torch.optim.SGD with the update done by one native multi-tensor kernel.

Same hyper-parameters, same ``state['momentum_buffer']`` entries (state dicts interchange with
``torch.optim.SGD``), same fp32 arithmetic per element (csrc/kernels/optim.hip).  The kernel
can also write the bf16 working copies of :class:`~grace_amd.parallel.precision.BF16Weights`
in the same pass, replacing ``BF16Weights.refresh()`` -- ``DistributedOptimizer(...,
weights=w)`` arranges that automatically.  CPU tensors (and ``GRACE_AMD_FORCE_TORCH=1``) run
``torch.optim.SGD``'s own functional update.

The learning rate and momentum are read from ``param_groups`` on every ``step()`` call; inside
a captured HIP graph they are frozen at capture time (as for any host scalar), so LR schedules
need eager steps or a re-capture.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
from torch.optim import SGD

from ..ops import _native


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense (contiguous up to a permutation of dims, e.g. channels_last)."""
    if t.is_contiguous():
        return True
    expected = 1
    for d in sorted(range(t.dim()), key=lambda d: t.stride(d)):
        if t.size(d) != 1 and t.stride(d) != expected:
            return False
        expected *= t.size(d)
    return True


def _same_layout(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Same memory image: equal shapes and equal strides on every dim of size > 1 (a 1x1 conv
    weight in channels_last and its contiguous bucket view differ only on size-1 dims)."""
    return a.shape == b.shape and all(sa == sb for sa, sb, n in zip(a.stride(), b.stride(), a.shape) if n > 1)


class FusedSGD(SGD):
    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, *,
                 maximize: bool = False):
        super().__init__(params, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                         nesterov=nesterov, maximize=maximize)
        self._working: Dict[int, torch.Tensor] = {}
        # the kernel honours the process-wide communication fault flag (parallel/health.py):
        # allocate it now, before any HIP-graph capture of the step
        devs = {p.device for g in self.param_groups for p in g["params"] if p.is_cuda}
        if devs:
            from . import health

            for d in sorted(devs, key=lambda d: d.index or 0):
                health.init(d)

    def attach_working_copies(self, weights) -> None:
        """Write ``weights``' bf16 working copies in the update kernel (BF16Weights)."""
        self._working = {id(master): work for _, _, master, work in weights.entries}

    @property
    def writes_working_copies(self) -> bool:
        return bool(self._working)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            native, rest = [], []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedSGD does not support sparse gradients")
                ok = (p.is_cuda and _native.native_on(p.device) and p.dtype == torch.float32
                      and p.grad.dtype == torch.float32 and _same_layout(p.grad, p)
                      and _dense(p))
                (native if ok else rest).append(p)
            if native:
                self._native_step(group, native)
            if rest:
                self._torch_step(group, rest)
        return loss

    def _native_step(self, group, params):
        mom = group["momentum"]
        first, later = [], []
        for p in params:
            st = self.state[p]
            if mom != 0 and st.get("momentum_buffer") is None:
                st["momentum_buffer"] = torch.empty_like(p)  # same strides as p
                first.append(p)
            else:
                later.append(p)
        # one launch per device (the kernel reads that device's communication fault word)
        devs = {}
        for ps, is_first in ((first, True), (later, False)):
            for p in ps:
                devs.setdefault((p.device, is_first), []).append(p)
        for (dev, is_first), ps in devs.items():
            bufs = [self.state[p].get("momentum_buffer") if mom != 0 else None for p in ps]
            w16 = [self._working_for(p) for p in ps]
            _native.lib().sgd_step(ps, [p.grad for p in ps], bufs, w16, float(group["lr"]), float(mom),
                                   float(group["dampening"]), float(group["weight_decay"]),
                                   bool(group["nesterov"]), bool(group.get("maximize", False)), is_first)
            for p, w in zip(ps, w16):  # working copies the kernel could not write (other strides)
                if w is None and id(p) in self._working:
                    self._working[id(p)].copy_(p)

    def _working_for(self, p) -> Optional[torch.Tensor]:
        w = self._working.get(id(p))
        return w if (w is not None and _same_layout(w, p)) else None

    def _torch_step(self, group, params):
        from torch.optim.sgd import sgd as functional_sgd

        bufs = [self.state[p].get("momentum_buffer") for p in params]
        functional_sgd(params, [p.grad for p in params], bufs, weight_decay=group["weight_decay"],
                       momentum=group["momentum"], lr=group["lr"], dampening=group["dampening"],
                       nesterov=group["nesterov"], maximize=group.get("maximize", False), foreach=False)
        if group["momentum"] != 0:
            for p, b in zip(params, bufs):
                self.state[p]["momentum_buffer"] = b
        for p in params:
            w = self._working.get(id(p))
            if w is not None:
                w.copy_(p)
