from ...compressor import QSGDCompressor  # noqa: F401
