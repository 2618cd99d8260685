from ...memory import DgcMemory  # noqa: F401
