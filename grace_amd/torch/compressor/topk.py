from ...compressor import TopKCompressor  # noqa: F401
