from ...communicator import Allgather  # noqa: F401
