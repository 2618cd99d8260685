"""grace_amd -- MI355X-native gradient compression for data-parallel training.

Same capabilities as GRACE (Crystal-wxy/grace): the Compressor / Memory / Communicator API,
every compression method, error feedback, and the Allreduce / Allgather / Broadcast
communicators -- with the compute in hand-written CDNA4 (gfx950) HIP kernels and the traffic
on RCCL over xGMI.

    from grace_amd import grace_from_params
    grc = grace_from_params({"compressor": "topk", "compress_ratio": 0.01,
                             "memory": "residual", "communicator": "allgather"})
    new_grad = grc.step(p.grad, name)
"""
__version__ = "0.1.0"

from .core import Communicator, Compressor, Memory, register_layout  # noqa: F401,E402
from .helper import grace_from_params  # noqa: F401,E402
