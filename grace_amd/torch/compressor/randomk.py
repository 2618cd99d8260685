from ...compressor import RandomKCompressor  # noqa: F401
