from ...communicator import Allreduce  # noqa: F401
