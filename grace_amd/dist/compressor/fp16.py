from ...compressor import FP16Compressor  # noqa: F401
