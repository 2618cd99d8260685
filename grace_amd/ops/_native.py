"""Loader for the native CDNA4 library ``grace_amd/_C.so``.

Policy (the framework must never silently run a slow path on the GPU):

* tensors on a GPU  -> the HIP kernel is REQUIRED; if ``_C.so`` is missing or fails to load we
  raise with the build command, we do not fall back to eager PyTorch.
* tensors on the CPU -> the pure-PyTorch reference implementation in each op module is used
  (it is also the numerics oracle the GPU tests compare against).

``GRACE_AMD_FORCE_TORCH=1`` switches GPU tensors to the PyTorch path explicitly (debug /
A-B timing only; never the default).
"""
from __future__ import annotations

import importlib
import os

import torch

_lib = None
_err: Exception | None = None


def lib():
    """Return the loaded native module or raise a descriptive error."""
    global _lib, _err
    if _lib is not None:
        return _lib
    if _err is not None:
        raise RuntimeError(
            "grace_amd native library is not available: "
            f"{_err!r}. Build it with `python -m grace_amd._build`."
        ) from _err
    try:
        import torch  # noqa: F401  (loads libamdhip64 / librccl from torch/lib first)

        alt = os.environ.get("GRACE_AMD_NATIVE_SO")  # e.g. the ASan preset build/asan/_C.so
        if alt:
            import sys
            from importlib import machinery, util

            spec = util.spec_from_loader("grace_amd._C", machinery.ExtensionFileLoader("grace_amd._C", alt))
            _lib = util.module_from_spec(spec)
            spec.loader.exec_module(_lib)
            sys.modules["grace_amd._C"] = _lib
        else:
            _lib = importlib.import_module("grace_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        _err = e
        return lib()
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except RuntimeError:
        return False


def use_native(t) -> bool:
    """True when ``t`` lives on a GPU and the native path must run."""
    if not getattr(t, "is_cuda", False):
        return False
    if os.environ.get("GRACE_AMD_FORCE_TORCH", "0") == "1":
        return False
    return True


def native_on(device) -> bool:
    """use_native() for a device instead of a tensor."""
    if torch.device(device).type != "cuda":
        return False
    return os.environ.get("GRACE_AMD_FORCE_TORCH", "0") != "1"
