from ...memory import PowerSGDMemory  # noqa: F401
