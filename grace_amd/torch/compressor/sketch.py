from ...compressor import SketchCompressor  # noqa: F401
