from ...compressor import SignSGDCompressor  # noqa: F401
