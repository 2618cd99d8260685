from ...compressor import EFSignSGDCompressor  # noqa: F401
