"""grace_amd.ops -- CDNA4 HIP kernels behind thin PyTorch wrappers.

Every op has two implementations:
  * the native HIP kernel in ``csrc/kernels/*.hip`` (used for GPU tensors, required there),
  * a plain PyTorch reference (used for CPU tensors and as the test oracle).
"""
from . import _native  # noqa: F401
from .layout import SegmentLayout, layout_for  # noqa: F401


def native_available() -> bool:
    return _native.available()


# the ``grace`` dispatcher operators (torch.ops.grace.*: csrc/ops_library.cpp + ops/library.py)
from . import library as _library  # noqa: E402

_library.register()
