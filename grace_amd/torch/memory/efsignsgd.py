from ...memory import EFSignSGDMemory  # noqa: F401
