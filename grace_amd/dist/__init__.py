"""Drop-in import paths for users of the reference's torch.distributed backend (grace_dl.dist).

``from grace_amd.dist.compressor.topk import TopKCompressor`` etc. resolve to the MI355X-native
implementations; the abstract base classes are the same objects as ``grace_amd.core``.
"""
from ..core import Communicator, Compressor, Memory  # noqa: F401
