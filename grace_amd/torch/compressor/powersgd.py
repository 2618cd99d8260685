from ...compressor import PowerSGDCompressor  # noqa: F401
