from ...communicator import Broadcast  # noqa: F401
