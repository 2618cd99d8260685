from ...memory import NoneMemory  # noqa: F401
