from ...compressor import OneBitCompressor  # noqa: F401
