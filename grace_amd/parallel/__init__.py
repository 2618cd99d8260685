"""Data-parallel integration: comm adapters, bucketed overlapped engine, DDP hook, optimizer."""
from .comm import LocalComm, TorchComm, default_comm, set_default_comm  # noqa: F401
from .ddp_hook import GraceDDPOptimizer, GraceHookState, grace_comm_hook  # noqa: F401
from .engine import GraceEngine  # noqa: F401
from .optimizer import DistributedOptimizer, broadcast_optimizer_state, broadcast_parameters  # noqa: F401
from .fused_sgd import FusedSGD  # noqa: F401
