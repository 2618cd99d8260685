"""bf16 working weights with fp32 masters (O2-style mixed precision) for the DP training step.

Under ``torch.autocast(bfloat16)`` every convolution / linear layer casts its fp32 weight to
bf16 in the forward pass and casts the bf16 weight gradient back to fp32 in the backward pass:
two small kernels per layer per step (~110 launches for ResNet-50, ~4.5 us of device time each
on MI355X).  :class:`BF16Weights` keeps the fp32 masters for the optimizer and the GRACE
buckets, and installs bf16 working copies in the modules:

* forward: autocast finds the weights already in bf16 -- no cast kernels;
* backward: the bf16 weight gradients are handed to the engine, whose gather kernel widens
  them into the fp32 gradient bucket (one launch per bucket, csrc/kernels/ef.hip);
* after ``optimizer.step()`` one batched cast kernel refreshes every working copy.

The numerics are those of autocast (weights rounded to bf16 with round-to-nearest-even, fp32
gradients and fp32 master update); only the launches differ.

    w = BF16Weights(model)                         # swaps the working copies in
    opt = DistributedOptimizer(SGD(w.master_parameters(model), ...), grc,
                               named_parameters=w.named_master_parameters(model), weights=w)
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Tuple

import torch
import torch.nn as nn

from ..ops import _native

DEFAULT_MODULES = (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.Linear)


class BF16Weights:
    def __init__(self, model: nn.Module, modules=DEFAULT_MODULES, dtype: torch.dtype = torch.bfloat16):
        if dtype != torch.bfloat16:
            raise ValueError("only bfloat16 working weights are supported")
        self.dtype = dtype
        # (module, attr, master fp32 Parameter, working bf16 Parameter)
        self.entries: List[Tuple[nn.Module, str, nn.Parameter, nn.Parameter]] = []
        self._master_of: Dict[int, nn.Parameter] = {}
        for m in model.modules():
            if not isinstance(m, modules):
                continue
            for attr in ("weight", "bias"):
                p = m._parameters.get(attr)
                if p is None or p.dtype != torch.float32:
                    continue
                work = nn.Parameter(torch.empty_like(p, dtype=dtype), requires_grad=p.requires_grad)
                m._parameters[attr] = work
                self.entries.append((m, attr, p, work))
                self._master_of[id(work)] = p
        self.refresh()

    # ------------------------------------------------------------------ parameter views
    @property
    def masters(self) -> List[nn.Parameter]:
        return [e[2] for e in self.entries]

    @property
    def working(self) -> List[nn.Parameter]:
        return [e[3] for e in self.entries]

    def named_master_parameters(self, model: nn.Module) -> Iterator[Tuple[str, nn.Parameter]]:
        """``model.named_parameters()`` with every working copy replaced by its fp32 master."""
        for n, p in model.named_parameters():
            yield n, self._master_of.get(id(p), p)

    def master_parameters(self, model: nn.Module) -> Iterator[nn.Parameter]:
        for _, p in self.named_master_parameters(model):
            yield p

    def grad_sources(self) -> Dict[int, nn.Parameter]:
        """id(master) -> the working parameter that receives its gradient in backward."""
        return {id(master): work for _, _, master, work in self.entries}

    # ------------------------------------------------------------------ updates
    @torch.no_grad()
    def refresh(self) -> None:
        """working <- bf16(master) for every layer (one batched kernel per 120 tensors)."""
        if not self.entries:
            return
        if self.entries[0][2].is_cuda and _native.native_on(self.entries[0][2].device):
            _native.lib().cast_segments_bf16([e[2] for e in self.entries], [e[3] for e in self.entries])
        else:
            for _, _, master, work in self.entries:
                work.copy_(master)

    def restore(self) -> None:
        """Put the fp32 masters back into the modules (e.g. before saving a plain checkpoint)."""
        for m, attr, master, _ in self.entries:
            m._parameters[attr] = master
        self.entries.clear()
        self._master_of.clear()
