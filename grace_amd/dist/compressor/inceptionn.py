from ...compressor import INCEPTIONNCompressor  # noqa: F401
