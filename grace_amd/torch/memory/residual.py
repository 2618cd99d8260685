from ...memory import ResidualMemory  # noqa: F401
