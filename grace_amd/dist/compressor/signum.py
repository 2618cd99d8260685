from ...compressor import SignumCompressor  # noqa: F401
