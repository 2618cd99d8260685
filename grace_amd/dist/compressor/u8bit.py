from ...compressor import U8bitCompressor  # noqa: F401
