"""``grace_amd.dist.helper.grace_from_params`` -- the torch.distributed factory with the
reference's dist defaults (/root/reference/grace_dl/dist/helper.py:1-86): compress_ratio 0.3,
lr 0.3, quantum_num 256, momentum 0.9 (Signum) / 0.3 (DGC memory), gradient clipping on,
compress_rank 1.  Deliberate fixes (survey 2.14): Threshold defaults to 0.01 (the reference's
256 selects nothing, #19), the clipping really is sqrt(allreduce(sum x^2)/W) (#2), PowerSGD and
Broadcast get the world size / rank (#3, #4), the efsignsgd memory exists (#13).  Explicit
keys always win."""
from __future__ import annotations

from typing import Any, Dict

from ..helper import grace_from_params as _factory

DIST_DEFAULTS: Dict[str, Any] = {
    "compress_ratio": 0.3,
    "lr": 0.3,
    "quantum_num": 256,
    "threshold": 0.01,
    "momentum": 0.9,
    "dgc_momentum": 0.3,
    "gradient_clipping": True,
    "compress_rank": 1,
}


def grace_from_params(params: Dict[str, Any], comm=None):
    p = dict(DIST_DEFAULTS)
    p.update(params)
    return _factory(p, comm=comm)
