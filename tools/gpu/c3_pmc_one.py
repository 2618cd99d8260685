"""One 3x3 implicit-GEMM direction of the f32 MFMA kernel, repeated: the program to hand to
``rocprofv3 --pmc`` (tools/gpu/r5_c3pmc.sh).
Usage: python tools/gpu/c3_pmc_one.py N C H W DIR TILE SPLITS [REPS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from grace_amd.ops import _native  # noqa: E402


def main():
    n, c, h, w, d, tile, splits = (int(a) for a in sys.argv[1:8])
    reps = int(sys.argv[8]) if len(sys.argv) > 8 else 10
    cl = torch.channels_last
    x = torch.randn(n, c, h, w, device="cuda").contiguous(memory_format=cl)
    wt = (torch.randn(c, c, 3, 3, device="cuda") * 0.05).contiguous(memory_format=cl)
    dy = torch.randn(n, c, h, w, device="cuda").contiguous(memory_format=cl)
    C = _native.lib()
    out = torch.empty_like(x) if d != 2 else torch.empty_like(wt)
    if tile < 0:  # MIOpen's data-gradient solver for the same problem (its zero fill included)
        def mi():
            return torch.ops.aten.convolution_backward(dy, x, wt, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                                       [True, False, False])[0]
        for _ in range(3):
            mi()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            mi()
        e.record()
        e.synchronize()
        print(f"miopen dgrad {n}x{c}x{h}x{w}: {s.elapsed_time(e) / reps * 1e3:.1f} us", flush=True)
        return
    for _ in range(reps):
        if d == 0:
            C.conv3x3_f32(0, x, wt, out, 1, splits, tile, None, 3)
        elif d == 1:
            C.conv3x3_f32(1, dy, wt, out, 1, splits, tile)
        else:
            C.conv3x3_f32(2, x, dy, out, 1, splits, tile, None, 3)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        if d == 1:
            C.conv3x3_f32(1, dy, wt, out, 1, splits, tile)
    e.record()
    e.synchronize()
    if d == 1:
        print(f"dgrad {n}x{c}x{h}x{w} tile {tile} splits {splits}: {s.elapsed_time(e) / reps * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
