"""Drop-in import paths for users of the reference's Horovod-PyTorch backend (grace_dl.torch).

``from grace_amd.torch.compressor.topk import TopKCompressor`` etc. resolve to the MI355X-native
implementations; the abstract base classes are the same objects as ``grace_amd.core``.
"""
from ..core import Communicator, Compressor, Memory  # noqa: F401
from ..parallel.optimizer import DistributedOptimizer, broadcast_optimizer_state, broadcast_parameters  # noqa: F401,E402
from .mpi_ops import (  # noqa: F401,E402
    allgather, allgather_async, allreduce, allreduce_, allreduce_async, allreduce_async_, broadcast, broadcast_,
    broadcast_async, broadcast_async_, init, is_initialized, local_rank, local_size, poll, rank, shutdown, size,
    synchronize)
