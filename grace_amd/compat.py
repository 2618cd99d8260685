"""Horovod-style ``Compression`` namespace (the reference's unused prototype API,
/root/reference/examples/dist/CIFAR10-dawndist/compression.py:560-567) mapped onto GRACE
compressors: ``Compression.none`` / ``Compression.fp16`` / ``Compression.bf16``."""
import torch

from .compressor import FP16Compressor, NoneCompressor


class Compression:
    none = NoneCompressor()
    fp16 = FP16Compressor(torch.float16)
    bf16 = FP16Compressor(torch.bfloat16)
