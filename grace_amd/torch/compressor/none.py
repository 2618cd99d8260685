from ...compressor import NoneCompressor  # noqa: F401
