from ...compressor import ThresholdCompressor  # noqa: F401
