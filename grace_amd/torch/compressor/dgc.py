from ...compressor import DgcCompressor  # noqa: F401
