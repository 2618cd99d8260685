"""Communicators (GRACE layer L4): Allreduce, Allgather, Broadcast."""
from .allgather import Allgather  # noqa: F401
from .allreduce import Allreduce  # noqa: F401
from .broadcast import Broadcast  # noqa: F401
