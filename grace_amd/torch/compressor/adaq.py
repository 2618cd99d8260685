from ...compressor import AdaqCompressor  # noqa: F401
