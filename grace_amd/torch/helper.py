"""``grace_amd.torch.helper.grace_from_params`` -- the Horovod-PyTorch factory's defaults
(/root/reference/grace_dl/torch/helper.py:1-80: compress_ratio 0.01, quantum_num 64,
threshold 0.01, lr 0.1, Signum momentum 0.9, DGC memory momentum 0.9 without clipping,
world_size = the job size).  The reference hard-codes these; here they are defaults and
explicit keys win."""
from __future__ import annotations

from typing import Any, Dict

from ..helper import grace_from_params as _factory

TORCH_DEFAULTS: Dict[str, Any] = {
    "compress_ratio": 0.01,
    "quantum_num": 64,
    "threshold": 0.01,
    "lr": 0.1,
    "momentum": 0.9,
    "dgc_momentum": 0.9,
    "gradient_clipping": False,
    "compress_rank": 1,
}


def grace_from_params(params: Dict[str, Any], comm=None):
    from .mpi_ops import size

    p = dict(TORCH_DEFAULTS)
    p.update(params)
    p.setdefault("world_size", size())
    return _factory(p, comm=comm)
