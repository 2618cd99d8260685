from ...compressor import TernGradCompressor  # noqa: F401
