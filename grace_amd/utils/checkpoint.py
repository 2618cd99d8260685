"""Checkpoint / resume including GRACE state.

The reference checkpoints only model/optimizer state through framework facilities in its
examples (tensorflow_mnist.py:149-163, keras ModelCheckpoint, hvd.broadcast_optimizer_state)
and never saves GRACE state -- error-feedback residuals, Signum/DGC momenta, PowerSGD Q and
Random-K step counters are silently lost on resume.  Here every component is Stateful, and
``save``/``load`` round-trip them together with the model and optimizer:

* the model / optimizer / ``extra`` go to ONE file written by rank 0 (data parallel: they are
  identical on every rank);
* GRACE state is PER RANK (each rank's residuals and momenta are its own; restoring rank 0's
  everywhere would turn the summed residual into W * r_0 and bias the first post-resume updates):
  with W > 1 every rank writes ``<path>.grace.rank<r>`` and reads back its own file
  (``per_rank=False`` forces the single-file layout, e.g. for W = 1);
* a ``DistributedOptimizer`` passed as ``optimizer`` is split: its base optimizer's state goes
  to the shared file, its engine's GRACE state is treated as above;
* bf16 working weights (``weights=`` a parallel.precision.BF16Weights): the fp32 MASTERS are
  saved under the parameter names (the module state_dict holds only the bf16 copies) and
  restored on load, then the working copies are refreshed from them;
* ``load`` uses ``torch.load(weights_only=True)`` (nothing executable is unpickled) and then
  broadcasts parameters from rank 0 so every replica restarts identical.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch
import torch.distributed as dist


def _dist() -> bool:
    return dist.is_available() and dist.is_initialized()


def _rank() -> int:
    return dist.get_rank() if _dist() else 0


def _world() -> int:
    return dist.get_world_size() if _dist() else 1


def grace_path(path: str, rank: Optional[int] = None) -> str:
    return f"{path}.grace.rank{_rank() if rank is None else rank}"


def _atomic_save(obj, path: str) -> None:
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(tmp)), exist_ok=True)
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _model_state(model: torch.nn.Module, weights=None) -> Dict[str, torch.Tensor]:
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    if weights is not None:  # fp32 masters instead of the bf16 working copies
        for n, p in weights.named_master_parameters(model):
            sd[n] = p.detach().cpu()
    return sd


def save(path: str, model: torch.nn.Module, optimizer=None, grace=None, extra: Optional[Dict[str, Any]] = None,
         per_rank: Optional[bool] = None, weights=None) -> None:
    """Collective when torch.distributed is initialised (ends with a barrier)."""
    per_rank = _world() > 1 if per_rank is None else per_rank
    grace, inner = _split(optimizer, grace)
    if _rank() == 0:
        state: Dict[str, Any] = {"model": _model_state(model, weights), "world_size": _world(),
                                 "grace_per_rank": bool(per_rank and grace is not None)}
        if inner is not None:
            state["optimizer"] = _cpu(inner.state_dict())
        if grace is not None and not per_rank:
            state["grace"] = _cpu(grace.state_dict())
        if extra:
            state["extra"] = extra
        _atomic_save(state, path)
    if per_rank and grace is not None:
        _atomic_save({"grace": _cpu(grace.state_dict()), "rank": _rank()}, grace_path(path))
    if _dist():
        dist.barrier()


def load(path: str, model: torch.nn.Module, optimizer=None, grace=None, per_rank: Optional[bool] = None,
         broadcast: bool = True, weights=None) -> Dict[str, Any]:
    state = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(state["model"])
    dev = next(model.parameters()).device
    if weights is not None:
        with torch.no_grad():
            for n, p in weights.named_master_parameters(model):
                if n in state["model"]:
                    p.copy_(state["model"][n])
        weights.refresh()
    grace, inner = _split(optimizer, grace)
    if inner is not None and "optimizer" in state:
        opt_sd = state["optimizer"]
        if inner is not optimizer and "optimizer" in opt_sd and "grace" in opt_sd:
            opt_sd = opt_sd["optimizer"]  # written by DistributedOptimizer.state_dict() directly
        inner.load_state_dict(_to(opt_sd, dev))
    if grace is not None:
        per_rank = state.get("grace_per_rank", False) if per_rank is None else per_rank
        if per_rank:
            saved_w = state.get("world_size", _world())
            if saved_w != _world():
                raise RuntimeError(f"per-rank GRACE state was saved at world size {saved_w}, loading at {_world()}")
            gs = torch.load(grace_path(path), map_location="cpu", weights_only=True)
            grace.load_state_dict(_to(gs["grace"], dev))
        elif "grace" in state:
            grace.load_state_dict(_to(state["grace"], dev))
    if broadcast and _dist():
        from ..parallel.optimizer import broadcast_parameters

        broadcast_parameters(model.state_dict(), root_rank=0)
    return state.get("extra", {})


def _split(optimizer, grace):
    """(GRACE state holder, plain optimizer): a DistributedOptimizer carries the GRACE state of
    its engine, which is per rank, next to the base optimizer's (replicated) state."""
    if optimizer is not None and hasattr(optimizer, "engine") and hasattr(optimizer, "_opt"):
        return (grace if grace is not None else optimizer.engine), optimizer._opt
    return grace, optimizer


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
