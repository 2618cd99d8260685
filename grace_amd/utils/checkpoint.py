"""Checkpoint / resume including GRACE state.

The reference checkpoints only model/optimizer state through framework facilities in its
examples (tensorflow_mnist.py:149-163, keras ModelCheckpoint, hvd.broadcast_optimizer_state)
and never saves GRACE state -- error-feedback residuals, Signum/DGC momenta, PowerSGD Q and
Random-K step counters are silently lost on resume.  Here every component is Stateful, and
``save``/``load`` round-trip them together with the model and optimizer:

* ``save`` writes on rank 0 only (one file) via torch.save of plain tensors/dicts;
* ``load`` uses ``torch.load(weights_only=True)`` (nothing executable is unpickled) and then
  broadcasts parameters from rank 0 so every replica restarts identical.
  Residuals are per-rank quantities: pass ``per_rank=True`` to save one file per rank.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def _path(path: str, per_rank: bool) -> str:
    return f"{path}.rank{_rank()}" if per_rank else path


def save(path: str, model: torch.nn.Module, optimizer=None, grace=None, extra: Optional[Dict[str, Any]] = None,
         per_rank: bool = False) -> None:
    if not per_rank and _rank() != 0:
        return
    state = {"model": {k: v.detach().cpu() for k, v in model.state_dict().items()}}
    if optimizer is not None:
        state["optimizer"] = _cpu(optimizer.state_dict())
    if grace is not None:
        state["grace"] = _cpu(grace.state_dict())
    if extra:
        state["extra"] = extra
    tmp = _path(path, per_rank) + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(tmp)), exist_ok=True)
    torch.save(state, tmp)
    os.replace(tmp, _path(path, per_rank))


def load(path: str, model: torch.nn.Module, optimizer=None, grace=None, per_rank: bool = False,
         broadcast: bool = True) -> Dict[str, Any]:
    state = torch.load(_path(path, per_rank), map_location="cpu", weights_only=True)
    model.load_state_dict(state["model"])
    if optimizer is not None and "optimizer" in state:
        optimizer.load_state_dict(_to(state["optimizer"], next(model.parameters()).device))
    if grace is not None and "grace" in state:
        grace.load_state_dict(_to(state["grace"], next(model.parameters()).device))
    if broadcast and dist.is_available() and dist.is_initialized():
        from ..parallel.optimizer import broadcast_parameters

        broadcast_parameters(model.state_dict(), root_rank=0)
    return state.get("extra", {})


def _cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj


def _to(obj, device):
    if isinstance(obj, torch.Tensor):
        return obj.to(device)
    if isinstance(obj, dict):
        return {k: _to(v, device) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to(v, device) for v in obj)
    return obj
