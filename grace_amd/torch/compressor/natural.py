from ...compressor import NaturalCompressor  # noqa: F401
