#!/usr/bin/env python3
"""Host-side AddressSanitizer pass over the native library's host code (CPU only).

Run through tools/asan_host_check.sh, which builds ``build/asan/_C.so`` (``python -m
grace_amd._build --asan``: every host translation unit instrumented, device code untouched),
preloads clang's ASan runtime and points ``GRACE_AMD_NATIVE_SO`` at the instrumented library.
Exercises what runs on the host without a GPU: module init / pybind registration, build info,
geometry helpers, and the argument-validation paths of the bindings (every TORCH_CHECK must
raise cleanly -- a bad shape must never reach pointer arithmetic).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from grace_amd.ops import _native  # noqa: E402


def expect_error(fn, *a):
    try:
        fn(*a)
    except (RuntimeError, TypeError, ValueError):
        return
    raise AssertionError(f"{fn} accepted invalid arguments")


def main():
    C = _native.lib()
    assert os.environ.get("GRACE_AMD_NATIVE_SO"), "run via tools/asan_host_check.sh"
    print(C.build_info())
    assert C.bn_supported(64) and not C.bn_supported(12)
    assert C.inceptionn_tiles(100_000) > 0
    uid = C.rccl_unique_id()
    assert len(uid) == 128
    cpu = torch.zeros(16)
    i32 = torch.zeros(16, dtype=torch.int32)
    expect_error(C.sparse_scatter_add, cpu, i32, cpu, 1.0, True)        # CPU tensors rejected
    expect_error(C.sparse_scatter_add_dev, cpu, i32, i32, cpu, 1.0, True)
    expect_error(C.threshold_compact, cpu, None, 0, 1.0, 1.0, 0.1, cpu, i32, i32, None)
    expect_error(C.bn_act_fwd, cpu.view(1, 16, 1, 1), None, None, None, None, None, None, 0.1, 1e-5, True)
    print("asan host check: OK")


if __name__ == "__main__":
    main()
